"""Per-dispatch view of one attack step from a rocprofv3 kernel trace (CSV): durations, grids and
the idle gaps between consecutive dispatches.  python scripts/trace_step.py <run_kernel_trace.csv> [step]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(ends) // 2
lo, hi = ends[k - 1] + 1, ends[k] + 1
step = rows[lo:hi]
t0 = int(step[0]["Start_Timestamp"])
busy = 0
prev_end = None
gap_total = 0
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0 if prev_end is None else s - prev_end
    gap_total += max(gap, 0)
    prev_end = e
    busy += e - s
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("phx::", "")
    grid = f'{int(r["Grid_Size_X"])//int(r["Workgroup_Size_X"])}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}'
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}us gap {gap / 1e3:6.1f} {grid:>14} vgpr {r['VGPR_Count']:>3} {name}")
span = int(step[-1]["End_Timestamp"]) - t0
print(f"step span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, gaps {gap_total / 1e6:.3f} ms, {len(step)} dispatches")

# per kernel family (template arguments kept) for the chosen step
agg = {}
for r in step:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("phx::", "")
    a = agg.setdefault(name, [0, 0])
    a[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    a[1] += 1
print("--- per kernel ---")
for name, (ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{ns / 1e6:8.3f} ms {n:5d} x {ns / n / 1e3:8.1f} us  {name}")
