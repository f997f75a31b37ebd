"""Diagnosis (GPU): which launch makes a concurrent step differ from the one-stream step?

PHX_CKSUM=1 makes phx_step_grad hash every tensor / statistics slot each op writes, right after
it, on its own stream.  This runs one one-stream step (PHX_CONC=0) as the reference and then N
concurrent steps on the same inputs, and prints, for every concurrent step that differs, the first
differing entries (launch order).  The first entry whose inputs agreed and whose output did not
names the kernel.

  python scripts/diag_cksum.py [model] [size] [dtype] [steps]
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

MODEL = sys.argv[1] if len(sys.argv) > 1 else "efficientdet-d4"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
DT = sys.argv[3] if len(sys.argv) > 3 else "bf16"
N = int(sys.argv[4]) if len(sys.argv) > 4 else 10
B = int(os.environ.get("DIAG_B", "4"))
imgs = torch.as_tensor(synth_images(list(range(B)), S)).cuda()
boxes = synth_boxes(list(range(B)), S)
v = EfficientDetVictim(MODEL, _well_conditioned_d4(S) if MODEL == "efficientdet-d4" else "synthetic", max_batch=B,
                       rng_seed=5, dtype=DT, image_size=S)
att = PatchAttacker(v, seed=7)


def step(conc: bool):
    os.environ["PHX_CONC"] = "1" if conc else "0"
    att.cur_step = 3
    att.call(imgs, boxes=boxes)
    torch.cuda.synchronize()
    ck = v.ctx.checksums(0)
    if conc:  # the first pass ran on the side executor: its entries follow the step's own
        ck = ck + v.ctx.checksums(1)
    return ck, att.grad.clone()


def changed_later(ck):
    post = {n[5:]: h for n, h in ck if n.startswith("post ")}
    return [n for n, h in ck if n in post and post[n] != h]


ref, g0 = step(False)
np.save(os.path.join("gpurun_out", f"g0_{os.environ.get('PHX_LIB', 'libphx.so')}.npy"), g0.cpu().numpy())
print("reference: tensors changed after their producer:", changed_later(ref)[:8])
print(f"{MODEL} {S} {DT} B={B}: {len(ref)} checksums per step", flush=True)
ndiff_steps = 0
for k in range(N):
    if k == 1:
        v.detect(imgs)
        torch.cuda.synchronize()
    got, g = step(True)
    rd = dict(ref)
    common = [(i, n, h) for i, (n, h) in enumerate(got) if n in rd]
    if k == 0:
        print(f"  concurrent step: {len(got)} checksums, {len(common)} shared with the one-stream step", flush=True)
    diffs = [(i, n, h) for i, n, h in common if rd[n] != h]
    same_grad = torch.equal(g, g0)
    moved = changed_later(got)
    if moved:
        print(f"  step {k}: {len(moved)} tensors changed after their producer:" +
              "".join(f"\n      {n}" for n in moved[:12]), flush=True)
    if not diffs:
        print(f"step {k}: identical (grad equal {same_grad})", flush=True)
        continue
    ndiff_steps += 1
    print(f"step {k}: {len(diffs)} entries differ (grad equal {same_grad}); first in launch order:", flush=True)
    for i, n, h in diffs[:8]:
        print(f"    [{i}] {n}  {rd[n]} -> {h}")
ref2, g2 = step(False)
print("one-stream rerun identical to the reference:", ref2 == ref and torch.equal(g2, g0))
print(f"differing concurrent steps: {ndiff_steps} / {N}")
