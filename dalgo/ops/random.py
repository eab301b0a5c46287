"""Counter-based random generation (csrc/kernels/random.hip) and K6 Monte-Carlo pi.

Every value is a pure function of (seed, stream, global index), so a rank that
generates rows [lo, hi) of a global matrix gets exactly the rows a single
process would: synthetic datasets are invariant to the world size.
"""
from __future__ import annotations

import numpy as np
import torch

from dalgo.ops import _ext
from dalgo.utils import philox

UNIFORM, NORMAL = 0, 1


def _values_cpu(seed, stream, idx: np.ndarray, dist: int, a: float, b: float) -> np.ndarray:
    if dist == UNIFORM:
        return (np.float32(a) + np.float32(b - a) * philox.uniform01(seed, stream, idx)).astype(np.float32)
    idx = np.asarray(idx, dtype=np.uint64)
    blk = idx >> np.uint64(1)
    c0 = (blk & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    c1 = (blk >> np.uint64(32)).astype(np.uint32)
    c2 = np.full(idx.shape, stream & 0xFFFFFFFF, dtype=np.uint32)
    c3 = np.full(idx.shape, (stream >> 32) & 0xFFFFFFFF, dtype=np.uint32)
    x, y, z, w = philox.philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    odd = (idx & np.uint64(1)).astype(bool)
    p = np.where(odd, z, x)
    q = np.where(odd, w, y)
    u1 = ((p >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)
    th = np.float32(6.283185307179586) * ((q >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0))
    return (np.float32(a) + np.float32(b) * np.sqrt(-2.0 * np.log(u1)) * np.cos(th)).astype(np.float32)


def philox_fill_(out: torch.Tensor, *, D: int | None = None, row_offset: int = 0, seed: int = 0,
                 stream: int = 0, dist: int = UNIFORM, a: float = 0.0, b: float = 1.0) -> torch.Tensor:
    """Fill a contiguous 2-D tensor: out[r, c] = value((row_offset + r) * D + c) for c < D, else 0."""
    if out.dim() == 1:
        out2 = out.view(-1, 1) if D is None or D == 1 else out.view(-1, D)
    else:
        out2 = out
    D = out2.shape[1] if D is None else int(D)
    if out2.is_cuda:
        _ext.ops().philox_fill(out2, D, int(row_offset), int(seed), int(stream), int(dist),
                               float(a), float(b))
        return out
    nrows, ld = out2.shape
    r = np.arange(nrows, dtype=np.int64).reshape(-1, 1) + row_offset
    c = np.arange(D, dtype=np.int64).reshape(1, -1)
    vals = _values_cpu(seed, stream, (r * D + c).reshape(-1), dist, a, b).reshape(nrows, D)
    out2.zero_()
    out2[:, :D] = torch.from_numpy(vals).to(out2.dtype)
    return out


def mc_pi_count(n: int, *, seed: int = 0, stream: int = 0, offset: int = 0,
                device: torch.device | str = "cpu") -> torch.Tensor:
    """Number of the points [offset, offset+n) of the stream that fall in the unit disc."""
    device = torch.device(device)
    if device.type == "cuda":
        cnt = torch.zeros(1, dtype=torch.int64, device=device)
        _ext.ops().mc_pi(int(seed), int(stream), int(offset), int(n), cnt)
        return cnt
    # CPU mirror of K6: point i = slot i % 3 of Philox block i / 3 (21-bit coordinates)
    if offset % 3:
        raise ValueError("offset must be a multiple of 3 (point triples share a Philox block)")
    total = 0
    chunk = 3 << 21
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        i = np.arange(offset + s, offset + s + m, dtype=np.uint64)
        blk = i // np.uint64(3)
        slot = (i % np.uint64(3)).astype(np.int64)
        c0 = (blk & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        c1 = (blk >> np.uint64(32)).astype(np.uint32)
        c2 = np.full(i.shape, stream & 0xFFFFFFFF, dtype=np.uint32)
        c3 = np.full(i.shape, (stream >> 32) & 0xFFFFFFFF, dtype=np.uint32)
        x, y, z, w = philox.philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
        sh, lo11, lo10 = np.uint32(11), np.uint32(0x7FF), np.uint32(0x3FF)
        u2 = (x & lo11) | ((y & lo10) << sh)
        v2 = (z & lo11) | ((w & lo10) << sh)
        u = np.where(slot == 0, x >> sh, np.where(slot == 1, z >> sh, u2))
        v = np.where(slot == 0, y >> sh, np.where(slot == 1, w >> sh, v2))
        scale = np.float32(2.0 / 2097152.0)
        fx = (u.astype(np.float32) + np.float32(0.5)) * scale - np.float32(1.0)
        fy = (v.astype(np.float32) + np.float32(0.5)) * scale - np.float32(1.0)
        total += int(np.count_nonzero(fx * fx + fy * fy <= np.float32(1.0)))
    return torch.tensor([total], dtype=torch.int64)
