"""HBM bytes per step from two rocprofv3 PMC passes over a whole bench run (scripts/gpu_r06_pmcstep.sh):
2 * FETCH_SIZE + WRITE_SIZE (KiB counters; gfx950 counts half the bytes of 16-B-per-lane reads,
MI355X_MICROARCH.md HBM section), summed over every dispatch and divided by the steps the run made.

  python tools/pmc_step.py <fetch dir> <write dir> <steps> [--kinds]"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    out = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            out[(r["Dispatch_Id"], r["Kernel_Name"].split("(")[0])] += float(r["Counter_Value"]) * 1024.0
    return out


fe, wr, steps = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE"), float(sys.argv[3])
tot = (2 * sum(fe.values()) + sum(wr.values())) / steps
print(f"HBM bytes per step: {tot / 1e9:.3f} GB (fetch x2 {2 * sum(fe.values()) / steps / 1e9:.3f}, write "
      f"{sum(wr.values()) / steps / 1e9:.3f})")
by = defaultdict(float)
for (did, name), v in fe.items():
    by[name] += 2 * v / steps
for (did, name), v in wr.items():
    by[name] += v / steps
for name, v in sorted(by.items(), key=lambda kv: -kv[1])[:25]:
    print(f"  {v / 1e6:9.1f} MB  {name[-90:]}")
