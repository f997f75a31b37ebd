"""Per-kernel summary of a rocprofv3 kernel trace stored as a rocpd SQLite database.

    python tools/rocpd_stats.py gpurun_out/prof_x/run_results.db [other.db] [--top 30] [--steps 12]

Prints calls, total / average duration per kernel name (template arguments kept, so GEMM variants
stay apart), the whole-trace kernel time, and — with two databases — the per-kernel difference.
--steps divides calls and totals to per-step figures (warmup + timed steps of the profiled bench).
"""
import argparse
import sqlite3
from collections import defaultdict


def load(path):
    c = sqlite3.connect(path)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    agg = defaultdict(lambda: [0, 0.0])
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        n = names.get(kid, str(kid)).split("(")[0]
        if n.startswith("void "):
            n = n[5:]
        a = agg[n]
        a[0] += 1
        a[1] += (e - s) / 1e3  # us
    return dict(agg)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=float, default=1.0)
    a = ap.parse_args()
    runs = [load(p) for p in a.db]
    base = runs[0]
    tot = [sum(v[1] for v in r.values()) / a.steps for r in runs]
    cnt = [sum(v[0] for v in r.values()) / a.steps for r in runs]
    print("kernel time per step (us): " + "  ".join(f"{t:.1f}" for t in tot) +
          "   launches per step: " + "  ".join(f"{c:.0f}" for c in cnt))
    keys = sorted(set().union(*runs), key=lambda k: -max(r.get(k, [0, 0])[1] for r in runs))
    for k in keys[:a.top]:
        cols = []
        for r in runs:
            n, t = r.get(k, [0, 0.0])
            cols.append(f"{n / a.steps:7.1f} {t / a.steps:9.1f} {t / max(n, 1):8.2f}")
        d = ""
        if len(runs) > 1:
            d = f"  d={(runs[-1].get(k, [0, 0])[1] - base.get(k, [0, 0])[1]) / a.steps:+8.1f}"
        print(" | ".join(cols) + d + "  " + k[:110])


if __name__ == "__main__":
    main()
