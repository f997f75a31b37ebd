"""GPU idle time of a kernel trace (rocprofv3 --kernel-trace CSV): the union of all kernels' [start,
end) intervals over every stream, over the last `--last` microseconds of the trace; prints the total
busy / idle time and the largest idle gaps with the kernels either side.

  python tools/idle_gaps.py <kernel_trace.csv> [--last 50000] [--top 25]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=float, default=50000.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-70:])
            for r in csv.DictReader(open(a.trace))]
    rows.sort()
    t_end = max(r[1] for r in rows)
    t0 = t_end - int(a.last * 1000)
    rows = [r for r in rows if r[0] >= t0]
    gaps, busy = [], 0
    cur_s, cur_e, last_name = rows[0][0], rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(((s - cur_e) / 1000, last_name, n, (cur_e - rows[0][0]) / 1000))
            cur_s, cur_e = s, e
        elif e > cur_e:
            cur_e = e
        if e >= cur_e:
            last_name = n
    busy += cur_e - cur_s
    span = (cur_e - rows[0][0]) / 1000
    idle = sum(g[0] for g in gaps)
    print(f"window {span:.1f} us, {len(rows)} kernels, busy {busy / 1000:.1f} us, idle {idle:.1f} us "
          f"in {len(gaps)} gaps ({sum(1 for g in gaps if g[0] > 5)} over 5 us: "
          f"{sum(g[0] for g in gaps if g[0] > 5):.1f} us)")
    for g in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g[0]:8.1f} us at {g[3]:9.1f}  after {g[1]}  before {g[2]}")


if __name__ == "__main__":
    main()
