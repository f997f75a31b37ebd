"""Summarise tools/gemm_bench GEMM_SWEEP output: best time per (shape, tile config) over split
counts, the overall best, and the configuration the current planner picks (its default run).

    python tools/sweep_table.py gpurun_out/gemm_sweep_m1.txt
"""
import collections
import re
import sys

CFGS = ['411', '412', '413', '415', '222', '212', '211', '111']


def main():
    rows = collections.OrderedDict()
    default = {}
    for line in open(sys.argv[1]):
        m = re.match(r'sweep M=\s*(\d+) N=\s*(\d+) K=\s*(\d+) cfg=(\d+) splits=(\d+)\s+([\d.]+)', line)
        if m:
            M, N, K, c, s, t = m.groups()
            rows.setdefault((int(M), int(N), int(K)), {})[(c, int(s))] = float(t)
            continue
        m = re.match(r'impl2 M=\s*(\d+) N=\s*(\d+) K=\s*(\d+) stats=\d\s+([\d.]+) us.*grid=(\d+)x(\d+)x(\d+)', line)
        if m:
            default[(int(m.group(1)), int(m.group(2)), int(m.group(3)))] = float(m.group(4))
    print('%-20s' % 'shape' + ''.join('%8s' % c for c in CFGS) + '   best')
    for k, v in rows.items():
        line = '%-20s' % ('%dx%dx%d' % k)
        for c in CFGS:
            ts = [t for (cc, s), t in v.items() if cc == c]
            line += '%8.1f' % (min(ts) if ts else 0)
        (bc, bs), bt = min(v.items(), key=lambda kv: kv[1])
        print(line, '  %s/%d %.1f' % (bc, bs, bt))


if __name__ == '__main__':
    main()
