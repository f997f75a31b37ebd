"""Compare tools/gemm_bench sweep results with the configuration plan_gemm2 picks (a Python port of
g2_pick + the half-row cascade + the split-K rule, fp32).  usage: python tools/sweep_pick.py sweep.txt"""
import re
import sys


def cdiv(a, b):
    return -(-a // b)


def pick(N, K, new=True):
    if N <= 32: c = (4, 1, 1)
    elif N <= 64: c = (4, 1, 2)
    elif N <= 96: c = (4, 1, 3)
    elif N <= 128: c = (2, 2, 2)
    elif N <= 160: c = (4, 1, 5)
    elif new and N % 128 and N % 96 == 0: c = (4, 1, 3)
    elif new and N % 128 and N % 160 == 0: c = (4, 1, 5)
    elif new and N >= 512 and K <= 64: c = (2, 1, 2)
    else: c = (2, 2, 2)
    return c


def plan(M, N, K, new=True):
    c = pick(N, K, new)
    bm = lambda q: q[0] * q[1] * 32
    bn = lambda q: (4 // q[0]) * q[2] * 32
    wgs = lambda q: cdiv(M, bm(q)) * cdiv(N, bn(q))
    if not (wgs(c) < 256 and K >= 256):
        if c == (4, 1, 2) and wgs(c) < 512: c = (2, 1, 1)
        if c == (2, 2, 2) and wgs(c) < 512: c = (2, 1, 2)
        if c == (2, 1, 2) and wgs(c) < 512: c = (1, 1, 1)
    tiles = cdiv(M, bm(c)) * cdiv(N, bn(c))
    splits = 1
    if tiles < 256 and K >= 256:
        splits = max(1, min(cdiv(512, tiles), K // 128))
    kslice = cdiv(cdiv(K, splits), 16) * 16
    splits = cdiv(K, kslice)
    return "%d%d%d" % c, splits


res = {}
for line in open(sys.argv[1]):
    m = re.match(r"sweep M=\s*(\d+) N=\s*(\d+) K=\s*(\d+) cfg=(\d+) splits=(\d+)\s+([\d.]+) us", line)
    if m:
        M, N, K, cfg, sp, us = int(m[1]), int(m[2]), int(m[3]), m[4], int(m[5]), float(m[6])
        res.setdefault((M, N, K), {})[(cfg, sp)] = us
tot_p = tot_b = 0
for (M, N, K), d in res.items():
    p = plan(M, N, K)
    best = min(d, key=d.get)
    tp = d.get(p, float("nan"))
    tot_p += tp if tp == tp else 0
    tot_b += d[best]
    print(f"M={M:8d} N={N:5d} K={K:5d} planned {p[0]} s{p[1]} {tp:8.1f} us  best {best[0]} s{best[1]} {d[best]:8.1f} us  {tp / d[best]:.2f}x")
print(f"planned total {tot_p:.1f} us, best total {tot_b:.1f} us")
