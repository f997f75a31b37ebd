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
from bench import PEAK_FP32_TFLOPS, kernel_roofline, synth_images  # noqa: E402

DEF_KINDS = {
    "unet_conv": "k_conv3_small<NT,MODE,VEC> (+ k_gemm2 MODE 4, the implicit-im2col GEMM, for the 64-128-channel "
                 "levels): 3x3 convs, transposed convs and their data gradients",
    "unet_wgrad": "k_wgrad_mfma<SRC,VEC> + column-sum bias gradients",
    "unet_bn": "k_colred64 statistics / BN-backward sums + BN apply",
    "unet_gemm": "k_gemm2 (attention 1x1 convs)",
}


def cpu_baseline(victim, d, S, budget_s=20.0):
    """The oracle's restatement of the defender step (PyTorch-CPU fp32: frozen D0 first pass, Masker,
    U-Net forward + every variable's gradient) on one image, timed on rank 0's host cores."""
    import numpy as np
    from mladversarialobjectdetection_amd import weights as W
    from oracle import defender as DF
    threads = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    wd = W.unpack(victim.manifest, victim.blob)
    params = d.params.cpu().numpy()
    mv = d.moving_statistics()
    moving = {b["name"]: (mv[b["moving_mean"]:b["moving_mean"] + b["channels"]],
                          mv[b["moving_variance"]:b["moving_variance"] + b["channels"]]) for b in d.manifest["bn"]}
    imgs = synth_images([0], S)
    n, t0 = 0, time.perf_counter()
    while True:
        DF.defender_step(params, moving, imgs, victim_weights=wd, seed=3, step=n, dtype=torch.float32)
        n += 1
        if time.perf_counter() - t0 > budget_s or n >= 50:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle restatement (PyTorch-CPU fp32) of the defender step, D0 + U-Net {S}x{S}, "
                      f"batch 1, {n} step(s), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--person-bias", type=float, default=4.6)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="run each step's first pass in the step (default: the fit loop hands train_step the next "
                         "batch, whose first pass then runs beside the current step's U-Net work)")
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
    # two batches, alternating (the generator's next batch is the other one)
    batches = [torch.as_tensor(synth_images(list(range((2 * rank + j) * B, (2 * rank + j + 1) * B)), S), device=dev)
               for j in range(2)]
    k = 0

    def train_step():
        nonlocal k
        out = d.train_step(batches[k % 2], next_inputs=None if a.no_prefetch else batches[(k + 1) % 2])
        k += 1
        return out

    for _ in range(a.warmup):
        train_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = train_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    el = float(dt.item())
    roofline = step_roof = None
    if not a.no_profile:
        # one extra, untimed step with per-launch-group HIP events (the victim context's profiler
        # covers the first pass, the Masker and every U-Net launch group)
        victim.ctx.profile(True)
        train_step()
        d.sync()
        rep = victim.ctx.profile_report()
        victim.ctx.profile(False)
        kind, r = max(rep.items(), key=lambda kv: kv[1]["ms"])
        # PMC traffic of the C5 configuration (512^2, 8 images): profiles/pmc_traffic_defender.json
        c5 = a.image_size == 512 and a.batch == 8
        roofline = kernel_roofline(kind, r, pmc="pmc_traffic_defender.json" if c5 else None)
        roofline["kernels"] = DEF_KINDS.get(kind, kind)
        fl = sum(v["flops"] for v in rep.values())
        step_roof = {"achieved_tflops_per_gpu": round(fl / (el / a.steps) / 1e12, 3),
                     "frac_fp32_peak": round(fl / (el / a.steps) / 1e12 / PEAK_FP32_TFLOPS, 4),
                     "algorithmic_gflop_per_step": round(fl / 1e9, 2),
                     "roofline_ms_per_step": round(sum(v["roof_ms"] for v in rep.values()), 3),
                     "breakdown_ms": {k: round(v["ms"], 3) for k, v in sorted(rep.items(), key=lambda kv: -kv[1]["ms"])}}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(victim, d, S)
    if rank == 0:
        print(json.dumps({
            "metric": "defender images/sec (attention U-Net 512px fwd+wgrad, frozen D0 first pass)",
            "value": round(world * B * a.steps / el, 3), "unit": "images/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * el / a.steps, 3),
            "higher_is_better": True, "scaling": "weak", "dtype": "f32",
            "data": f"synthetic (two alternating U(-1,1) batches, synthetic efficientdet-d0 weights, person_bias "
                    f"{a.person_bias}); first pass " + ("in the step" if a.no_prefetch else
                                                        "of the next batch beside each step (phx_def_set_next)"),
            "config": {"workload": f"C5: defender {S}x{S}, {B} images/GPU", "global_batch": world * B,
                       "u_net_params": d.handle.num_params, "loss": float(out["loss"].item()),
                       "parallelism": f"dp{world}"},
            "roofline": roofline, "step_roofline": step_roof, "cpu_baseline": cpu}))


if __name__ == "__main__":
    main()
