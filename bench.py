"""Benchmark: patch-optimisation images/sec (EfficientDet-D0 512px fwd+bwd) — BASELINE.json metric.

One "step" = PatchAttacker.train_step on one batch: first (clean) victim pass + pre_nms + soft-NMS,
EOT paste, second victim pass, loss, victim data-gradient, EOT backward, RCCL all-reduce of
[d patch | d scale] (N>1), Adam + clip.  Workload = BASELINE config C2/C3: D0 512x512, 16 images
per GPU, fp32, bn=local (batch statistics per rank), synthetic data: U(-1,1) images keyed by global
image index, 1-3 injected person boxes per image for placement (the first pass still runs in full),
synthetic weights (seed 0).

  python bench.py                       # N=1
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# multiply-adds per image forward at the model's native size (efficientdet_arch_test.py:47-114);
# one step = clean fwd + attack fwd + attack dgrad = 3 forward-equivalents, 2 FLOP per MAC
# (SURVEY.md 8d); other image sizes scale with the pixel count
MACS = {"efficientdet-d0": (512, 2_532_997_127), "efficientdet-d1": (640, 6_095_640_824),
        "efficientdet-d2": (768, 10_986_053_156), "efficientdet-d3": (896, 24_869_554_579),
        "efficientdet-d4": (1024, 55_146_068_329), "efficientdet-lite0": (320, 977_617_221),
        "efficientdet-lite4": (640, 20_221_443_966)}
D0_MACS = MACS["efficientdet-d0"][1]
FLOP_PER_IMAGE = 3 * 2 * D0_MACS
PEAK_FP32_TFLOPS = 157.3   # MI355X fp32 matrix / vector peak (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
# environment knobs that skip kernels (timing diagnostics only; a build without PHX_DEBUG_KNOBS ignores
# them): a line measured with one set would not be the reference's step
WORK_SKIPPING_KNOBS = ("PHX_SKIP_TIMING", "PHX_SKIP_KINDS", "PHX_NO_DROP")


def flop_per_image(model, size):
    native, macs = MACS.get(model, (512, D0_MACS))
    return 3 * 2 * macs * (size / native) ** 2


def synth_images(global_idx, size):
    out = np.empty((len(global_idx), size, size, 3), np.float32)
    for i, g in enumerate(global_idx):
        out[i] = np.random.default_rng(1234 + g).uniform(-1, 1, (size, size, 3))
    return out


def synth_boxes(global_idx, size):
    """1 + (g mod 3) person boxes, height U(96,384), aspect w/h U(.35,.6), inside the image."""
    res = []
    for g in global_idx:
        r = np.random.default_rng(99 + g)
        bx = []
        for _ in range(1 + g % 3):
            h = r.uniform(96, 384) * size / 512
            w = h * r.uniform(0.35, 0.6)
            y0 = r.uniform(0, size - h)
            x0 = r.uniform(0, size - w)
            bx.append([y0, x0, y0 + h, x0 + w])
        res.append(np.asarray(bx, np.float32))
    return res


def cpu_baseline(size, batch, threads, budget_s=15.0):
    """The oracle's restatement of the same step (PyTorch-CPU fp32) on a bounded sample."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    from oracle import step as ST
    torch.set_num_threads(threads)
    ctx = _lib.Context("efficientdet-d0", size, 1)
    man = ctx.manifest()
    wd = W.unpack(man, W.synthetic_blob(man, seed=0))
    idx = list(range(batch))
    imgs = synth_images(idx, size)
    boxes = synth_boxes(idx, size)
    patch = np.random.default_rng(7).uniform(-1, 1, (640, 640, 3)).astype(np.float32)
    n, t0 = 0, time.perf_counter()
    while True:
        ST.attack_step(wd, imgs, patch, 0.4, boxes=boxes, seed=0, step=n, image_size=size, dtype=torch.float32)
        n += 1
        if time.perf_counter() - t0 > budget_s or n >= 100:
            break
    dt = time.perf_counter() - t0
    return {"value": round(batch * n / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle restatement (PyTorch-CPU fp32), D0 {size}x{size}, batch {batch}, {n} step(s), {dt:.1f} s"}


# kernels behind each launch-group kind of the library profiler (for the rocprof cross-check)
KIND_KERNELS = {
    "gemm": "k_gemm2 / k_gemm2r <WM,TM,TN,MODE,SK,NS,BF,ST>, k_gemm2k <TM,TN,MODE,SK,BF,ST> (deep K: K split "
            "across a workgroup's waves) (+ k_gemm<NT,WM,MODE,SK> for N<=16, k_gemm_splitk_reduce(_stats))",
    "bn_stats": "k_bn_finalize<false,StatsEpi,NS> (statistics partials from the producer's epilogue)",
    "bn_bwd_reduce": "k_bn_finalize<true,BwdEpi2,NS> (BN-backward sums from the consumer's dgrad)",
    "dw_fwd": "k_dw_fwd<K,S,RPT,STATS,NS>",
    "dw_bwd": "k_dw_bwd<K,S,RPT,GS,NS>",
    "sep_fwd": "k_sep_fwd<C,NS,XV,STATS,PT> (depthwise 3x3 -> pointwise MFMA + bias + BN statistics, one launch)",
    "sep_bwd": "k_sep_bwd<C,NS,GS,YBF> (pointwise dgrad on MFMA over the window + depthwise transpose)",
}


def pmc_traffic(kind, fname="pmc_traffic.json"):
    """HBM bytes per launch of `kind` from a committed rocprofv3 PMC summary of this configuration
    (FETCH_SIZE x2 for gfx950's half-counted wide reads + WRITE_SIZE, MI355X_MICROARCH.md HBM
    section; scripts/pmc_summary.py), or None."""
    p = os.path.join(ROOT, "profiles", fname)
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get("kinds", {}).get(kind)
    return None if e is None else e.get("bytes_per_launch")


def kernel_roofline(kind, r, mfma_peak=PEAK_FP32_TFLOPS, pmc="pmc_traffic.json"):
    """Roofline of the dominant launch group: its bound is the one whose peak-time for the group's
    algorithmic work is larger; achieved = algorithmic bytes (FLOPs) / measured time."""
    sec = r["ms"] * 1e-3
    hbm_bound = r.get("hbm_ms", 0.0) >= r.get("mfma_ms", 0.0)
    if hbm_bound:
        ach, peak, unit, bound = r["bytes"] / sec / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"
    else:
        ach, peak, unit, bound = r["flops"] / sec / 1e12, mfma_peak, "TFLOP/s", "mfma"
    out = {"bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
           "traffic": pmc_traffic(kind, pmc) if pmc else None, "kernel": kind, "kernels": KIND_KERNELS.get(kind, kind),
           "launches": r["count"], "avg_us": round(1e3 * r["ms"] / r["count"], 2),
           "algorithmic_bytes_per_launch": round(r["bytes"] / r["count"]),
           "algorithmic_flops_per_launch": round(r["flops"] / r["count"]),
           "roofline_time_frac": round(r.get("roof_ms", 0.0) / r["ms"], 4) if r["ms"] else None}
    return out


def _lib_path():
    from mladversarialobjectdetection_amd import _lib
    return _lib.LIB_PATH


def _lib_digest():
    import hashlib
    with open(_lib_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 steps of C2 take ~2.8 s: long enough for the driver's GPU-busy sampler to see the run
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=2)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--model", default="efficientdet-d0",
                    help="victim (the headline metric is D0; others for the secondary configs)")
    ap.add_argument("--placement", choices=("injected", "first-pass"), default="injected",
                    help="injected: 1-3 synthetic person boxes per image (SURVEY.md 8d); first-pass: the "
                         "reference's own flow, patches go onto the first pass's soft-NMS boxes")
    ap.add_argument("--dtype", choices=("f32", "bf16"), default="f32",
                    help="1x1-conv arithmetic: f32 (the reference's precision, configs C1-C3) or bf16 "
                         "(C4: bf16 matrix cores, fp32 accumulation)")
    ap.add_argument("--person-bias", type=float, default=0.0,
                    help="lift the person class-logit bias so the clean pass yields real soft-NMS candidates")
    ap.add_argument("--draw", choices=("auto", "standard", "well-conditioned"), default="auto",
                    help="synthetic weight draw: standard = SURVEY.md 8d; well-conditioned = weights.WELL_CONDITIONED "
                         "(the draw test_bf16_d4_1024_four_images validates C4 on); auto = well-conditioned for "
                         "D4 bf16, standard otherwise")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary line (the reference's own placement flow, measured after the headline)")
    args = ap.parse_args()

    # the line certifies itself: every PHX_* knob of the run goes into it, and the diagnostics that
    # skip work (wrong results; compiled out of the shipped library) refuse to run
    phx_env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("PHX_")}
    bad = [k for k in WORK_SKIPPING_KNOBS if k in phx_env]
    if bad:
        sys.exit(f"bench.py: {', '.join(bad)} set -- these skip work and give wrong results; no headline")

    from mladversarialobjectdetection_amd import distributed as ddp
    ddp.init_from_env()
    rank, world = ddp.rank(), ddp.world()
    # one rank per GPU; ranks beyond the visible GPUs share them (a rehearsal of the N>1 path on a
    # one-GPU box with PHX_DIST_BACKEND=gloo — never the case on a real node)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker, _pad_boxes
    B, S = args.batch, args.image_size
    draw = args.draw
    if draw == "auto":
        draw = "well-conditioned" if (args.model == "efficientdet-d4" and args.dtype == "bf16") else "standard"
    if draw == "well-conditioned":
        # the parity test's configuration: its weights, its EOT key (rng_seed 5), its images and boxes
        from mladversarialobjectdetection_amd import _lib
        from mladversarialobjectdetection_amd import weights as wmod
        wts = wmod.well_conditioned_blob(_lib.Context(args.model, S, 1).manifest())
        victim = EfficientDetVictim(args.model, wts, image_size=S, max_batch=B, rng_seed=5, device=local,
                                    dtype=args.dtype)
    else:
        victim = EfficientDetVictim(args.model, "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=0,
                                    device=local, person_bias=args.person_bias, dtype=args.dtype)
    att = PatchAttacker(victim, seed=7, device=dev)
    gidx = list(range(rank * B, (rank + 1) * B))
    images = torch.as_tensor(synth_images(gidx, S), device=dev)
    # injected placement boxes, resident on the device like the images ([B,maxb,4] + counts)
    boxes = _pad_boxes(synth_boxes(gidx, S), B, dev) if args.placement == "injected" else None
    # first-pass placement: two alternating batches, each step handed the next (phx_set_next: its
    # first pass runs beside the step), as the secondary line below
    fp_batches = None if boxes is not None else [
        images, torch.as_tensor(synth_images(list(range(B * (world + rank), B * (world + rank + 1))), S), device=dev)]
    k_main = 0

    def main_step():
        nonlocal k_main
        if fp_batches is None:
            att.train_step(images, boxes=boxes)
        else:
            att.train_step(fp_batches[k_main % 2], next_inputs=fp_batches[(k_main + 1) % 2])
        k_main += 1

    for _ in range(args.warmup):
        main_step()
    torch.cuda.synchronize()
    # (after a step: with injected boxes the concurrent first pass holds its own executor)
    ws_gb = victim.ctx.workspace_bytes(B) / 1e9
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        main_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(dt.item())
    images_per_s = world * B * args.steps / elapsed

    patches_headline = att.step_metrics()["patches"] if rank == 0 else 0

    # the step's one collective timed alone (N>1): the same [d patch | d scale | metric row] payload,
    # on a copy, between barriers, max over ranks — so a scaling curve separates the exchange from
    # the per-rank compute
    allreduce = None
    if world > 1:
        buf = att._red.clone()
        n_ar = 20
        ddp.allreduce_sum_(buf)  # warm the communicator
        torch.cuda.synchronize()
        torch.distributed.barrier()
        ta = time.perf_counter()
        for _ in range(n_ar):
            ddp.allreduce_sum_(buf)
        torch.cuda.synchronize()
        da = torch.tensor([time.perf_counter() - ta], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(da, op=torch.distributed.ReduceOp.MAX)
        ar_ms = 1e3 * float(da.item()) / n_ar
        nbytes = buf.numel() * buf.element_size()
        allreduce = {"ms_per_call": round(ar_ms, 4), "bytes": nbytes, "calls_per_step": 1,
                     "backend": str(torch.distributed.get_backend()),
                     "algbw_GBps": round(nbytes / (ar_ms * 1e-3) / 1e9, 3),
                     # ring all-reduce moves 2 (N-1)/N of the payload over each rank's links
                     "busbw_GBps": round(2 * (world - 1) / world * nbytes / (ar_ms * 1e-3) / 1e9, 3),
                     "frac_of_step": round(ar_ms / (1e3 * elapsed / args.steps), 4)}
        del buf

    roofline = None
    step_roof = None
    if not args.no_profile:
        # one extra, untimed step with per-launch-group HIP events on the launch stream
        victim.ctx.profile(True)
        main_step()
        rep = victim.ctx.profile_report()
        victim.ctx.profile(False)
        kind, r = max(rep.items(), key=lambda kv: kv[1]["ms"])
        mpeak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_FP32_TFLOPS
        # committed PMC traffic summaries: C2 (pmc_traffic.json) and C4 (pmc_traffic_d4bf16.json)
        cfg = (args.model, args.dtype, S, B)
        pmc = {("efficientdet-d0", "f32", 512, 16): "pmc_traffic.json",
               ("efficientdet-d4", "bf16", 1024, 4): "pmc_traffic_d4bf16.json"}.get(cfg)
        roofline = kernel_roofline(kind, r, mpeak, pmc=pmc)
        step_ach = flop_per_image(args.model, S) * images_per_s / world / 1e12
        step_roof = {"achieved_tflops_per_gpu": round(step_ach, 3),
                     "frac_mfma_peak": round(step_ach / mpeak, 4), "mfma_peak_tflops": mpeak,
                     "breakdown_ms": {k: round(v["ms"], 3) for k, v in sorted(rep.items(), key=lambda kv: -kv[1]["ms"])}}
        # bandwidth-aware conv roofline: sum over launches of max(bytes/HBM, flops/MFMA)
        roof_ms = sum(v.get("roof_ms", 0.0) for v in rep.values())
        step_roof["roofline_ms_per_step"] = round(roof_ms, 3)
        step_roof["frac_of_roofline"] = round(roof_ms / (1e3 * elapsed / args.steps), 4)

    # secondary line (not `value`): the same workload with the reference's placement flow — patches
    # on the first pass's soft-NMS person boxes (attacker.py:180-184) with a person prior that gives
    # ~1500 patches per step — timed the same way on a fresh victim after the headline
    secondary = None
    if not args.no_secondary and args.placement == "injected" and args.model == "efficientdet-d0":
        del att
        torch.cuda.empty_cache()
        v2 = EfficientDetVictim(args.model, "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=0,
                                device=local, person_bias=4.6, dtype=args.dtype)
        a2 = PatchAttacker(v2, seed=7, device=dev)
        # at least 20 timed steps whatever --steps is (the driver's --steps 20 gave 5 before)
        steps2 = max(20, args.steps // 4)
        # two batches, alternating; the fit loop hands each step the next one, whose first pass
        # then runs beside the step's second pass and backward (phx_set_next)
        batches = [images, torch.as_tensor(synth_images(list(range(B * (world + rank), B * (world + rank + 1))), S),
                                           device=dev)]
        k2 = 0

        def step2():
            nonlocal k2
            a2.train_step(batches[k2 % 2], next_inputs=batches[(k2 + 1) % 2])
            k2 += 1

        for _ in range(args.warmup):
            step2()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t1 = time.perf_counter()
        for _ in range(steps2):
            step2()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        d2 = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        if world > 1:
            torch.distributed.all_reduce(d2, op=torch.distributed.ReduceOp.MAX)
        e2 = float(d2.item())
        m2 = a2.step_metrics()
        secondary = {"placement": "first-pass", "person_bias": 4.6, "steps": steps2,
                     "first_pass": "the next batch's, beside each step (phx_set_next); two alternating batches",
                     "value": round(world * B * steps2 / e2, 3), "unit": "images/s",
                     "ms_per_step": round(1e3 * e2 / steps2, 3), "patches_per_step": int(m2["patches"])}
        att = a2

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "efficientdet-d0":
        threads = min(16, len(os.sched_getaffinity(0)))
        cpu = cpu_baseline(S, args.cpu_batch, threads)

    if rank == 0:
        met = att.step_metrics() if secondary is None else {"patches": patches_headline}
        line = {
            "metric": "patch-opt images/sec (EffDet-D0 512px fwd+bwd)" if args.model == "efficientdet-d0"
                      else f"patch-opt images/sec ({args.model} {S}px fwd+bwd)",
            "value": round(images_per_s, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": ("synthetic (U(-1,1) images, " + ("1-3 injected person boxes/image" if boxes is not None else
                     "placement from the first pass's soft-NMS boxes") + f", synthetic {args.model} weights"
                     + (f", person_bias {args.person_bias}" if args.person_bias and draw == "standard" else "")
                     + (", well-conditioned draw (gamma U(0.2,0.4), beta N(1,0.1), person prior 3, EOT key 5): "
                        "the configuration test_bf16_d4_1024_four_images checks" if draw == "well-conditioned"
                        else "") + ")"),
            "config": {"workload": (f"C{2 if world == 1 else 3}: EfficientDet-D0" if args.model == "efficientdet-d0"
                                    else ("C4: " if args.model == "efficientdet-d4" else "") + args.model)
                                   + f" patch attack {S}x{S}, "
                                   f"{B} images/GPU, bn=local", "global_batch": world * B, "image_size": S,
                       "workspace_gb_per_gpu": round(ws_gb, 3), "placement": args.placement,
                       "patches_per_step": int(met["patches"]),
                       "parallelism": f"dp{world}"},
            "roofline": roofline,
            "step_roofline": step_roof,
            "cpu_baseline": cpu,
            "allreduce": allreduce,
            "secondary": secondary,
            "env": phx_env,
            "library": {"so": os.path.relpath(_lib_path(), ROOT), "sha256_16": _lib_digest()},
        }
        print(json.dumps(line))


if __name__ == "__main__":
    main()
