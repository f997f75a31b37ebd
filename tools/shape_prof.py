"""Per-shape launch-group timing of one attack step (PHX_PROF_DETAIL=1 + the library profiler):
prints every (kind, shape) group with its time, launches and achieved bandwidth / FLOP rate.

  PHX_PROF_DETAIL=1 python tools/shape_prof.py [--model efficientdet-d0] [--batch 16] [--dtype f32]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PHX_PROF_DETAIL", "1")

from bench import synth_boxes, synth_images  # noqa: E402
from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker, _pad_boxes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="efficientdet-d0")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--image-size", type=int, default=0)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    v = EfficientDetVictim(a.model, "synthetic", seed=0, image_size=a.image_size, max_batch=a.batch, dtype=a.dtype)
    S = v.ctx.image_size
    idx = list(range(a.batch))
    imgs = torch.as_tensor(synth_images(idx, S)).cuda()
    boxes = _pad_boxes(synth_boxes(idx, S), a.batch, imgs.device)
    att = PatchAttacker(v, seed=7)
    for _ in range(3):
        att.train_step(imgs, boxes=boxes)
    torch.cuda.synchronize()
    v.ctx.profile(True)
    att.train_step(imgs, boxes=boxes)
    rep = v.ctx.profile_report()
    v.ctx.profile(False)
    tot = sum(r["ms"] for r in rep.values())
    print(f"{a.model} {S}px B={a.batch} {a.dtype}: {tot:.3f} ms in {sum(r['count'] for r in rep.values())} groups")
    rows = sorted(rep.items(), key=lambda kv: -kv[1]["ms"])[:a.top]
    for k, r in rows:
        us = 1e3 * r["ms"] / r["count"]
        gbs = r["bytes"] / (r["ms"] * 1e-3) / 1e9 if r["ms"] else 0
        tfs = r["flops"] / (r["ms"] * 1e-3) / 1e12 if r["ms"] else 0
        roof = r.get("roof_ms", 0) / r["ms"] if r["ms"] else 0
        print(f"{r['ms']*1e3:8.1f} us {r['count']:4d}x {us:7.1f} us {gbs:7.0f} GB/s {tfs:7.2f} TF/s roof {roof:5.2f}  {k}")


if __name__ == "__main__":
    main()
