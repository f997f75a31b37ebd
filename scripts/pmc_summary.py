"""Summarise rocprofv3 PMC passes (scripts/gpu_pmc.sh) into per-kind HBM traffic per launch.

HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (both in KiB), per MI355X_MICROARCH.md's HBM section: on gfx950
FETCH_SIZE counts exactly half the bytes of wide (16 B/lane) coalesced reads; WRITE_SIZE is exact for
16-B stores.  Kinds match the library profiler's launch groups; `launches` counts the group's primary
kernel.

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/pmc_traffic.json [set] [source]

set: "detector" (default; the attack step's kinds) or "defender" (tools/defender_bench.py's U-Net kinds).
"""
import csv
import json
import re
import sys
from collections import defaultdict

KINDS = [  # (kind, substring, primary?) — first match wins
    ("gemm", "k_gemm_splitk_reduce", False), ("gemm", "k_gemm2<", True), ("gemm", "k_gemm2r<", True),
    ("gemm", "k_gemm2k<", True), ("gemm", "k_gemm<", True),
    ("dw_fwd", "k_dw_fwd<", True), ("dw_bwd", "k_dw_bwd<", True),
    ("sep_fwd", "k_sep_fwd<", True), ("sep_bwd", "k_sep_bwd<", True),
    ("bn_stats", "k_bn_finalize<false", True),
    ("bn_stats", "k_colred_part<phx::StatsAcc", True), ("bn_stats", "k_colred_final<phx::StatsEpi>", False),
    ("bn_bwd_reduce", "k_bn_finalize<true", True),
    ("bn_bwd_reduce", "k_colred_part<phx::BwdAcc", True), ("bn_bwd_reduce", "k_colred_final<phx::BwdEpi2>", False),
    ("se_bwd", "k_se_mlp_bwd", False), ("se_bwd", "k_ew_gstats<phx::SeBwdApply", True),
    ("se", "k_se_mlp", False), ("se", "k_colred_part<phx::SumAcc", True),
]


# the defender step: U-Net 3x3 convs (implicit-gather GEMMs are k_gemm2 MODE 4, the template's 4th
# argument), weight gradients, BN reductions; regex patterns start with "re:"
DEF_KINDS = [
    ("unet_conv", "k_conv3_small<", True), ("unet_conv", r"re:k_gemm2<\d+, \d+, \d+, 4,", True),
    ("unet_conv", "k_im2col", False),
    ("unet_wgrad", "k_wgrad_mfma<", True), ("unet_wgrad", "k_wgrad_fold", False),
    ("unet_bn", "k_colred64", True), ("unet_bn", "k_un_bn_final", False), ("unet_bn", "k_un_bnb_final", False),
    ("unet_bn", "k_un_bnb_apply", False), ("unet_bn", "k_un_bnact", False),
    ("soft_nms", "k_soft_nms", True),
]


def kind_of(name, kinds=None):
    for k, sub, prim in (kinds or KINDS):
        if sub.startswith("re:") and re.search(sub[3:], name) or not sub.startswith("re:") and sub in name:
            return k, prim
    return None, False


def load(d, counter):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    out = {}
    for r in rows:
        if r["Counter_Name"] == counter:
            out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
    return out


def main(fd, wd, dst, kset="detector", source=None):
    kinds_tab = DEF_KINDS if kset == "defender" else KINDS
    f, w = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    agg = defaultdict(lambda: {"launches": 0, "fetch_kib": 0.0, "write_kib": 0.0})
    per_kernel = defaultdict(lambda: {"n": 0, "fetch_kib": 0.0})
    for did, (name, v) in f.items():
        k, prim = kind_of(name, kinds_tab)
        per_kernel[name]["n"] += 1
        per_kernel[name]["fetch_kib"] += v
        if k is None:
            continue
        agg[k]["fetch_kib"] += v
        agg[k]["launches"] += int(prim)
    # the two passes are separate runs of the same deterministic program: match by kernel order
    for did, (name, v) in w.items():
        k, _ = kind_of(name, kinds_tab)
        if k is not None:
            agg[k]["write_kib"] += v
        per_kernel[name].setdefault("write_kib", 0.0)
        per_kernel[name]["write_kib"] = per_kernel[name].get("write_kib", 0.0) + v
    kinds = {}
    for k, a in agg.items():
        byt = (2.0 * a["fetch_kib"] + a["write_kib"]) * 1024.0
        kinds[k] = {"launches": a["launches"], "hbm_bytes": byt,
                    "bytes_per_launch": round(byt / max(1, a["launches"])),
                    "read_bytes": 2.0 * a["fetch_kib"] * 1024.0, "write_bytes": a["write_kib"] * 1024.0}
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), " +
                     (source or "python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile"),
           "correction": "bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB), gfx950 half-counted wide reads",
           "kinds": kinds}
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    with open(dst.replace(".json", "_kernels.csv"), "w") as fh:
        fh.write("kernel,dispatches,fetch_kib_x2,write_kib\n")
        for name, a in sorted(per_kernel.items(), key=lambda kv: -kv[1]["fetch_kib"]):
            fh.write(f"\"{name[:120]}\",{a['n']},{2 * a['fetch_kib']:.1f},{a.get('write_kib', 0.0):.1f}\n")
    for k, v in sorted(kinds.items()):
        print(f"{k:14s} launches {v['launches']:5d}  MB/launch {v['bytes_per_launch'] / 1e6:9.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:6])
