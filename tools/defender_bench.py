"""Defender-step throughput (BASELINE config C5): PatchAttackDefender.train_step
= frozen D0 first pass (inference BN) + soft-NMS, Masker EOT (self-supervised patches), attention
U-Net forward + weight gradient, one SUM all-reduce of [d variables | loss] at world > 1, Adam.
Synthetic U(-1,1) images, synthetic victim weights with the person prior lifted so the first pass
yields real placement boxes, U-Net initialised as generator.py does.  C5 is 64 images over 8 GPUs:
8 images per GPU is the default.  Prints one JSON line.

    python tools/defender_bench.py [--batch 8] [--steps 10] [--warmup 2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/defender_bench.py
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import synth_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--person-bias", type=float, default=4.6)
    a = ap.parse_args()

    from mladversarialobjectdetection_amd import distributed as ddp
    ddp.init_from_env()
    rank, world = ddp.rank(), ddp.world()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    B, S = a.batch, a.image_size
    victim = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=0,
                                device=local, person_bias=a.person_bias)
    d = PatchAttackDefender(victim, protege_config_override={"nms_configs": {"iou_thresh": .5, "score_thresh": .5}},
                            seed=3, device=dev)
    images = torch.as_tensor(synth_images(list(range(rank * B, (rank + 1) * B)), S), device=dev)
    for _ in range(a.warmup):
        d.train_step(images)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = d.train_step(images)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    el = float(dt.item())
    if rank == 0:
        print(json.dumps({
            "metric": "defender images/sec (attention U-Net 512px fwd+wgrad, frozen D0 first pass)",
            "value": round(world * B * a.steps / el, 3), "unit": "images/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * el / a.steps, 3),
            "higher_is_better": True, "scaling": "weak", "dtype": "f32",
            "data": f"synthetic (U(-1,1) images, synthetic efficientdet-d0 weights, person_bias {a.person_bias})",
            "config": {"workload": f"C5: defender {S}x{S}, {B} images/GPU", "global_batch": world * B,
                       "u_net_params": d.handle.num_params, "loss": float(out["loss"].item()),
                       "parallelism": f"dp{world}"}}))


if __name__ == "__main__":
    main()
