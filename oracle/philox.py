"""Philox4x32-10 (Salmon et al., SC'11) in numpy — mirrors csrc/common.hpp bit for bit.

Counter layout used by the product (csrc/kernels_eot.hip):
    ctr = (c0, c1 = box slot, c2 = global image index, c3 = step << 8 | stream)
    key = (seed & 0xffffffff, seed >> 32)
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

RNG_PRINT, RNG_PLACE, RNG_BOX, RNG_NOISE, RNG_DROP, RNG_AUG = 1, 2, 3, 4, 5, 6


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over broadcastable uint32 counters; returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (x.astype(np.uint32) for x in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def u01(v):
    """[0,1) from the top 24 bits, exact in float32."""
    return (np.asarray(v, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def u01_open0(v):
    return ((np.asarray(v, dtype=np.uint32) >> np.uint32(8)) + np.uint32(1)).astype(np.float32) * np.float32(
        1.0 / 16777216.0)


def runif(v, lo, hi):
    """tf.random.uniform(minval, maxval): u * (maxval - minval) + minval, fp32 ops."""
    lo = np.float32(lo)
    hi = np.float32(hi)
    return (u01(v) * (hi - lo)).astype(np.float32) + lo


def rnorm(a, b, mean, sd):
    """tf.random.normal: z * stddev + mean with a Box-Muller z (fp32)."""
    u1 = u01_open0(a)
    u2 = u01(b)
    z = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)
    return (z.astype(np.float32) * np.float32(sd)).astype(np.float32) + np.float32(mean)


def draw(seed, c0, c1, c2, step, stream):
    c3 = np.uint32(((int(step) << 8) | int(stream)) & 0xFFFFFFFF)
    return philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
