"""Compare two rocprofv3 kernel-stats CSVs per kernel (total time per call-normalised step)."""
import csv
import re
import sys


def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("phx::", "")
        a = d.setdefault(n, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"]) / 1e3
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
ta, tb = sum(v[1] for v in a.values()), sum(v[1] for v in b.values())
print(f"total {ta:.0f} us -> {tb:.0f} us")
rows = []
for k in set(a) | set(b):
    x, y = a.get(k, [0, 0.0]), b.get(k, [0, 0.0])
    rows.append((y[1] - x[1], k, x, y))
for dlt, k, x, y in sorted(rows)[:15] + sorted(rows)[-8:]:
    print(f"{dlt:9.0f} us  {x[1]:8.0f} -> {y[1]:8.0f}  ({x[0]}/{y[0]} calls)  {k}")
