"""Average duration per (kernel, grid) of a rocprofv3 kernel-trace CSV, for kernels matching a pattern.
  python tools/kt_summary.py run_kernel_trace.csv [pattern]"""
import collections
import csv
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if pat in n:
        d[(n.split("(")[0][-70:], r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / len(v):9.2f} us x{len(v):4d} tot {sum(v):9.1f}  {k[0]}  grid {k[1]}")
