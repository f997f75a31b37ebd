"""Diagnosis (GPU): how does a residual add's output differ in a concurrent step?

Runs a one-stream reference step (PHX_CONC=0) with PHX_CKSUM=1, copies every second-pass add's
inputs and output (raw storage), then concurrent steps; for each concurrent step whose first
differing checksum is a second-pass add, prints where in the tensor the output differs.
"""
import os
import sys

import numpy as np
import torch

os.environ["PHX_CKSUM"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from bench import synth_boxes, synth_images  # noqa: E402
from test_gpu_bf16 import _well_conditioned_d4  # noqa: E402
from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker  # noqa: E402

S, B, N = 1024, 4, int(sys.argv[1]) if len(sys.argv) > 1 else 8
imgs = torch.as_tensor(synth_images(list(range(B)), S)).cuda()
boxes = synth_boxes(list(range(B)), S)
v = EfficientDetVictim("efficientdet-d4", _well_conditioned_d4(S), max_batch=B, rng_seed=5, dtype="bf16", image_size=S)
att = PatchAttacker(v, seed=7)
st = torch.cuda.current_stream().cuda_stream


def step(conc):
    os.environ["PHX_CONC"] = "1" if conc else "0"
    att.cur_step = 3
    att.call(imgs, boxes=boxes)
    torch.cuda.synchronize()
    return v.ctx.checksums(0)


def tensor(op, which, nbytes):
    t = torch.empty(nbytes // 2, dtype=torch.int16, device="cuda")
    v.ctx.call("phx_debug_tensor", 0, op, which, t.data_ptr(), nbytes, st)
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


ref = step(False)
adds = sorted({int(n.split()[2]) for n, _ in ref if n.startswith("p1 f ") and n.endswith(" add out")})
sizes = {}
for i in adds:
    for nb in range(0, 1 << 30):  # find the size from the error message once
        try:
            tensor(i, 0, 2)
        except Exception as e:  # noqa: BLE001
            nb = int(str(e).split("(")[-1].split(" bytes")[0])
        sizes[i] = nb
        break
refout = {i: tensor(i, 0, sizes[i]) for i in adds}
print(f"{len(adds)} second-pass adds; sizes (MB):", [round(sizes[i] / 1e6, 1) for i in adds[:6]], "...", flush=True)
rd = dict(ref)
for k in range(N):
    got = step(True)
    diffs = [n for n, h in got if n in rd and rd[n] != h]
    if not diffs:
        print(f"step {k}: identical", flush=True)
        continue
    first = diffs[0]
    print(f"step {k}: first differing {first}", flush=True)
    if not (first.startswith("p1 f ") and first.endswith(" add out")):
        continue
    i = int(first.split()[2])
    out = tensor(i, 0, sizes[i])
    r = refout[i]
    bad = np.nonzero(out != r)[0]
    nel = r.size
    # NHWC coordinates: find C from the op's program?  report flat ranges and 64-element (128-B) lines
    lines = np.unique(bad // 64)
    runs = np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1)
    print(f"    {bad.size} of {nel} elements differ in {lines.size} 128-B lines, {len(runs)} runs; "
          f"first {bad[:4].tolist()} last {bad[-2:].tolist()}; run lengths {sorted({len(x) for x in runs})[:12]}")
    f32 = lambda u: (u.astype(np.uint32) << 16).view(np.float32)  # noqa: E731
    a_in = tensor(i, 1, sizes[i])
    b_in = tensor(i, 2, sizes[i])
    t = torch.empty(sizes[i] // 2, dtype=torch.int16, device="cuda")
    v.ctx.call("phx_debug_tensor", 1, i, 0, t.data_ptr(), sizes[i], st)
    torch.cuda.synchronize()
    p0 = t.cpu().numpy().view(np.uint16)
    for j in bad[:8]:
        g, rr, av, bv, pv = (f32(x[j:j + 1])[0] for x in (out, r, a_in, b_in, p0))
        print(f"      [{j}] ref {rr:.6g} got {g:.6g} | a(raw) {av:.6g} b {bv:.6g} | got-b {g - bv:.6g} ref-b {rr - bv:.6g}"
              f" | first-pass out {pv:.6g}")
    print(f"      got == first-pass value at {int(np.sum(out[bad] == p0[bad]))} of {bad.size} bad elements; "
          f"got == b at {int(np.sum(out[bad] == b_in[bad]))}")
    # is the wrong value some other element of the reference (a stale or misplaced read)?
    w = f32(out[bad[:64]])
    rv = f32(r)
    hits = [int(np.nonzero(rv == x)[0][0]) if np.any(rv == x) else -1 for x in w[:8]]
    print(f"      wrong values found elsewhere in the reference tensor at: {hits}", flush=True)
