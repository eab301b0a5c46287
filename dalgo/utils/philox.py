"""NumPy mirror of the device Philox4x32-10 stream (csrc/include/dalgo/common.h).

``draw_u32(seed, stream, idx)`` returns exactly the 32-bit word the HIP kernels
use for index ``idx`` of stream ``stream`` under key ``seed``:

    philox4x32_10(counter = (idx >> 2) as 2x32 || stream as 2x32,
                  key     = seed as 2x32)[idx & 3]

Used by the CPU (gloo) reference path and by the numerics tests so sampling
decisions are bit-identical between CPU and GPU runs, for any sharding.
"""
from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 on uint32 arrays; returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & _MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & _MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return c0, c1, c2, c3


def draw_u32(seed: int, stream: int, idx) -> np.ndarray:
    """32-bit draws for integer indices ``idx`` (array-like of non-negative ints)."""
    idx = np.asarray(idx, dtype=np.uint64)
    blk = idx >> np.uint64(2)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    stream = int(stream) & 0xFFFFFFFFFFFFFFFF
    c0 = (blk & _MASK32).astype(np.uint32)
    c1 = (blk >> np.uint64(32)).astype(np.uint32)
    c2 = np.full(idx.shape, stream & 0xFFFFFFFF, dtype=np.uint32)
    c3 = np.full(idx.shape, stream >> 32, dtype=np.uint32)
    r = philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, seed >> 32)
    out = np.empty(idx.shape, dtype=np.uint32)
    lane = (idx & np.uint64(3)).astype(np.int64)
    for j in range(4):
        m = lane == j
        out[m] = r[j][m]
    return out


def frac_threshold(frac: float) -> int:
    """Bernoulli threshold: an index is selected iff draw < threshold (same as C++)."""
    if frac <= 0.0:
        return 0
    if frac >= 1.0:
        return 0xFFFFFFFF
    t = int(np.floor(frac * 4294967296.0))
    return min(t, 0xFFFFFFFF)


def bernoulli_mask(seed: int, stream: int, idx, frac: float) -> np.ndarray:
    """Selection mask used by every minibatch sampler (K7)."""
    idx = np.asarray(idx)
    if frac >= 1.0:
        return np.ones(idx.shape, dtype=bool)
    return draw_u32(seed, stream, idx) < np.uint32(frac_threshold(frac))


def uniform01(seed: int, stream: int, idx) -> np.ndarray:
    """Uniform floats in [0, 1) with 24-bit resolution (same mapping as the kernels)."""
    u = draw_u32(seed, stream, idx)
    return (u >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
