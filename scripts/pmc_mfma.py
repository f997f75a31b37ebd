"""Summarise the MFMA-busy PMC pass (scripts/gpu_pmc_mfma.sh) per kernel template.

mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024): the matrix-core busy cycles over
the SIMD-cycles the kernel held the chip for (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs x 4
SIMDs).  wait / issue / active: shares of SQ_WAVE_CYCLES (SQ_WAIT_ANY = parked on s_waitcnt or a
barrier; SQ_WAIT_INST_ANY = issue-stalled; SQ_ACTIVE_INST_ANY = issuing).

    python scripts/pmc_mfma.py gpurun_out/pmc_mfma_d0 [out.json]
"""
import collections
import csv
import json
import re
import sys


def main():
    d = sys.argv[1]
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        k = (r["Dispatch_Id"], r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for (_, name), c in per.items():
        t = re.sub(r"\(.*", "", name).replace("void ", "").replace("phx::", "")
        a = agg[t]
        a["launches"] += 1
        for kk, v in c.items():
            a[kk] += v
    out = {}
    for t, a in sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
        cyc = a["GRBM_GUI_ACTIVE"] / 8.0
        wave = max(a["SQ_WAVE_CYCLES"], 1.0)
        out[t] = {"launches": int(a["launches"]), "gpu_cycles": round(cyc),
                  "mfma_util": round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / max(cyc * 1024, 1.0), 4),
                  "wait": round(a["SQ_WAIT_ANY"] / wave, 3), "issue_stall": round(a["SQ_WAIT_INST_ANY"] / wave, 3),
                  "active": round(a["SQ_ACTIVE_INST_ANY"] / wave, 3),
                  "lds_bank_conflict_per_launch": round(a["SQ_LDS_BANK_CONFLICT"] / a["launches"])}
    for t, v in list(out.items())[:25]:
        print(f"{v['gpu_cycles']:>10} cyc  mfma {v['mfma_util']:6.3f}  wait {v['wait']:5.2f}  stall {v['issue_stall']:5.2f} "
              f" active {v['active']:5.2f}  ldsconf {v['lds_bank_conflict_per_launch']:>8}  x{v['launches']:<4} {t[:70]}")
    if len(sys.argv) > 2:
        json.dump({"source": d, "kernels": out}, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
