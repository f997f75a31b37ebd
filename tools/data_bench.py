"""Input-pipeline throughput: phx_letterbox + phx_augment on a batch of
decoded 640x480 uint8 photos-sized inputs into 512x512 canvases, device-resident inputs, timed
with HIP events on the launch stream; the oracle (numpy, cv2 restatement) times one image on the
host for scale.  Prints one JSON line.

    python tools/data_bench.py [--batch 64] [--iters 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mladversarialobjectdetection_amd import data as D  # noqa: E402
from mladversarialobjectdetection_amd.attacker import EfficientDetVictim  # noqa: E402

MEAN = [0.485 * 255, 0.456 * 255, 0.406 * 255]
STD = [0.229 * 255, 0.224 * 255, 0.225 * 255]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--src", default="480x640")
    ap.add_argument("--size", type=int, default=512)
    a = ap.parse_args()
    h, w = map(int, a.src.split("x"))
    S, B = a.size, a.batch
    v = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=128, max_batch=2)
    rng = np.random.default_rng(0)
    ims = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for _ in range(B)]
    dev = torch.device("cuda", 0)
    src, off, dims = D.pack_images(ims, dev)
    out = torch.empty((B, S, S, 3), device=dev)
    aug = torch.empty_like(out)
    mean = np.asarray(MEAN, np.float32)
    std = np.asarray(STD, np.float32)
    stream = torch.cuda.current_stream().cuda_stream

    def lb():
        v.ctx.call("phx_letterbox", src.data_ptr(), off.data_ptr(), dims.data_ptr(), B, mean.ctypes.data,
                   std.ctypes.data, S, S, out.data_ptr(), stream)

    def ag(i):
        v.ctx.call("phx_augment", out.data_ptr(), B, S, S, i, 0, aug.data_ptr(), stream)

    for i in range(3):
        lb()
        ag(i)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_lb = t_ag = 0.0
    for i in range(a.iters):
        e[0].record()
        lb()
        e[1].record()
        ag(i)
        e[2].record()
        e[2].synchronize()
        t_lb += e[0].elapsed_time(e[1])
        t_ag += e[1].elapsed_time(e[2])
    t_lb /= a.iters
    t_ag /= a.iters
    canvas = B * S * S * 3 * 4
    lb_bytes = B * h * w * 3 + canvas            # uint8 source read once + fp32 canvas written
    ag_bytes = 3 * canvas                         # sums read + apply read + write
    from oracle import data as OD
    t0 = time.perf_counter()
    OD.map_fn(ims[0], (S, S), MEAN, STD)
    cpu_one = time.perf_counter() - t0
    print(json.dumps({
        "metric": "input pipeline images/s (letterbox + augment)", "batch": B, "src": [h, w], "size": S,
        "images_per_s": round(B / ((t_lb + t_ag) * 1e-3), 1),
        "letterbox_ms": round(t_lb, 4), "augment_ms": round(t_ag, 4),
        "letterbox_gbs": round(lb_bytes / (t_lb * 1e-3) / 1e9, 1),
        "augment_gbs": round(ag_bytes / (t_ag * 1e-3) / 1e9, 1), "hbm_peak_gbs": 8000.0,
        "cpu_oracle_map_fn_images_per_s": round(1.0 / cpu_one, 2),
        "cpu_note": "oracle numpy restatement of _map_fn (float64, 1 image), not the reference's cv2"}))


if __name__ == "__main__":
    main()
