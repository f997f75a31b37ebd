"""Diagnostic (GPU box): why the D4 256^2 bf16 step's loss moves when the deep-K GEMMs switch from the
cross-workgroup split (k_gemm2 + reduce) to the wave-split-K kernel (k_gemm2k, PHX_GEMM_WSK_BF16=1)
(VERDICT r5 item 4).  test_bf16_d4_256_matches_emulation_oracle's draw and step.

    python scripts/diag_bf16_wsk_layers.py          (parent: CPU only; each plan runs in a child)

Runs, each in its own process (the plan switches are read once per process):
  A  PHX_GEMM_WSK_BF16=0 (bf16 deep-K GEMMs split across workgroups: the round-5 default)
  B  PHX_GEMM_WSK_BF16=1 (split across the waves of one workgroup instead: the default since round 6)
  C  A again (run-to-run determinism)
and, in the parent, the fp64 oracle with the product's bf16 rounding points (Bf16Conv1x1 /
Bf16Store) and the plain fp64 oracle.  Per batch norm (its input = the stored conv output, forward
order) it prints the fraction of elements where runs A and B differ, the largest difference in bf16
quanta of the larger magnitude (a quantum is 2^-7 of the value's binade), A and B's relative distance
and each run's relative distance from the emulation; then every run's per-image max scores, loss-anchor
indices and loss.  Work files live in /tmp on the box; the summary goes to stdout."""
import json
import os
import subprocess
import sys

import numpy as np

S4 = 256
TMP = "/tmp/bf16wsk"


def _child(tag):
    import torch
    sys.path.insert(0, os.getcwd())
    from bench import synth_boxes, synth_images
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    blob = W.well_conditioned_blob(_lib.Context("efficientdet-d4", S4, 1).manifest())
    v = EfficientDetVictim("efficientdet-d4", blob, image_size=S4, max_batch=2, rng_seed=5, dtype="bf16")
    imgs = synth_images([0, 1], S4)
    boxes = synth_boxes([0, 1], S4)
    att = PatchAttacker(v, seed=7)
    att.cur_step = 3
    att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
    st = torch.cuda.current_stream().cuda_stream
    m = torch.empty(2, device="cuda")
    anc = torch.empty(2, dtype=torch.int32, device="cuda")
    v.ctx.call("phx_debug_last_maxscores", m.data_ptr(), anc.data_ptr(), st)
    out = dict(loss=float(att.metrics_buf.cpu().numpy()[_lib.M_LOSS]), grad=att.grad.cpu().numpy(),
               m=m.cpu().numpy(), anchor=anc.cpu().numpy())
    if tag == "prep":
        np.savez(TMP + "_prep.npz", blob=blob, patch=att.patch.cpu().numpy(), imgs=imgs)
        with open(TMP + "_manifest.json", "w") as f:
            json.dump(v.manifest, f)
        with open(TMP + "_boxes.json", "w") as f:
            json.dump([b.tolist() for b in boxes], f)
        return
    shapes = json.load(open(TMP + "_shapes.json"))
    for name, shp in shapes.items():
        buf = torch.empty(int(np.prod(shp)), device="cuda")
        v.ctx.call("phx_debug_tap", name.encode(), 0, buf.data_ptr(), buf.numel(), st)
        out["tap:" + name] = buf.cpu().numpy().reshape(shp)
    np.savez(f"{TMP}_{tag}.npz", **out)


def _oracle():
    import torch
    sys.path.insert(0, os.getcwd())
    from mladversarialobjectdetection_amd import weights as W
    from oracle import detector as D
    from oracle import step as ST
    torch.set_num_threads(16)
    z = np.load(TMP + "_prep.npz")
    wd = W.unpack(json.load(open(TMP + "_manifest.json")), z["blob"].copy())
    boxes = [np.asarray(b, np.float32) for b in json.load(open(TMP + "_boxes.json"))]
    kw = dict(boxes=boxes, seed=5, step=3, image_size=S4, model="efficientdet-d4")
    orig = D.Detector.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.taps = {}
    D.Detector.__init__ = init
    try:
        rem = ST.attack_step(wd, z["imgs"], z["patch"], np.float32(0.4), bf16=True, **kw)
    finally:
        D.Detector.__init__ = orig
    bns = {e["name"][:-len("/gamma")] for e in json.load(open(TMP + "_manifest.json")) if e["name"].endswith("/gamma")}
    taps = {n: t[0].detach().permute(0, 2, 3, 1).numpy().astype(np.float32)
            for n, t in rem["det"].taps.items() if n in bns and t[0].dim() == 4}
    with open(TMP + "_shapes.json", "w") as f:
        json.dump({n: list(t.shape) for n, t in taps.items()}, f)
    r64 = ST.attack_step(wd, z["imgs"], z["patch"], np.float32(0.4), **kw)
    np.savez(TMP + "_emul.npz", loss=rem["loss"], grad=rem["grad"], m=rem["m"], loss64=r64["loss"],
             grad64=r64["grad"], m64=r64["m"], **{"tap:" + n: t for n, t in taps.items()})
    return list(taps)


def _quanta(a, b):
    """|a - b| in bf16 quanta of the larger magnitude (8-bit significand)."""
    mag = np.maximum(np.abs(a), np.abs(b)).astype(np.float64)
    q = np.exp2(np.floor(np.log2(np.maximum(mag, 1e-30))) - 7)
    return np.abs(a.astype(np.float64) - b) / q


def _rel(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / max(np.linalg.norm(b.astype(np.float64)), 1e-30))


def main():
    os.makedirs("/tmp", exist_ok=True)
    env0 = {k: v for k, v in os.environ.items() if not k.startswith("PHX_")}
    runs = {"A": {"PHX_GEMM_WSK_BF16": "0"}, "B": {"PHX_GEMM_WSK_BF16": "1"}, "C": {"PHX_GEMM_WSK_BF16": "0"}}

    def run(tag, extra):
        r = subprocess.run([sys.executable, __file__, "child", tag], env={**env0, **extra}, timeout=600)
        if r.returncode != 0:
            sys.exit(f"child {tag} failed ({r.returncode})")

    run("prep", {})
    names = _oracle()
    for tag, extra in runs.items():
        run(tag, extra)
    E = np.load(TMP + "_emul.npz")
    R = {t: np.load(f"{TMP}_{t}.npz") for t in runs}
    print(f"{'batch norm (input = stored conv output)':58s} {'A!=B':>8s} {'maxq':>5s} {'|A-B|':>9s} {'A!=C':>8s}"
          f" {'eA':>9s} {'eB':>9s}")
    first = None
    for n in names:
        e = E["tap:" + n]
        a, b, c = (R[t]["tap:" + n] for t in "ABC")
        dab, dac = float(np.mean(a != b)), float(np.mean(a != c))
        if first is None and dab > 0:
            first = n
        qab = float(_quanta(a, b).max()) if dab else 0.0
        print(f"{n[-58:]:58s} {dab:8.2e} {qab:5.1f} {_rel(b, a):9.3e} {dac:8.2e} {_rel(a, e):9.3e} {_rel(b, e):9.3e}")
    print(f"first layer where A and B differ: {first}")
    print(f"fp64 oracle: m {E['m64']} loss {float(E['loss64']):.7f}")
    print(f"emulation  : m {E['m']} loss {float(E['loss']):.7f}  |emul-fp64|/fp64 "
          f"{abs(float(E['loss']) - float(E['loss64'])) / abs(float(E['loss64'])):.2e}")
    for t in "ABC":
        r = R[t]
        g = r["grad"][:-1].astype(np.float64)
        print(f"run {t}: m {r['m']} anchors {r['anchor']} loss {float(r['loss']):.7f} "
              f"|gpu-fp64|/fp64 {abs(float(r['loss']) - float(E['loss64'])) / abs(float(E['loss64'])):.2e} "
              f"|gpu-emul|/emul {abs(float(r['loss']) - float(E['loss'])) / abs(float(E['loss'])):.2e} "
              f"d patch vs emul {_rel(g, E['grad'][:-1]):.3e} vs fp64 {_rel(g, E['grad64'][:-1]):.3e}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        _child(sys.argv[2])
    else:
        main()
