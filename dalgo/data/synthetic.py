"""On-device synthetic generators for the clustering and graph benchmarks."""
from __future__ import annotations

import torch

from dalgo.ops import random as drandom


def blob_centers(k: int, d: int, seed: int, device, spread: float = 10.0) -> torch.Tensor:
    C = torch.empty((k, d), dtype=torch.float32, device=device)
    drandom.philox_fill_(C, D=d, seed=seed, stream=21, dist=drandom.NORMAL, a=0.0, b=spread)
    return C


def blobs(n: int, d: int, k: int, *, row_range=None, device="cpu", dtype=torch.float32,
          seed: int = 0, spread: float = 10.0, noise: float = 1.0, chunk: int = 1 << 22) -> torch.Tensor:
    """Rows [lo, hi) of an n x d mixture of k isotropic Gaussians (index-keyed)."""
    lo, hi = row_range if row_range is not None else (0, n)
    device = torch.device(device)
    C = blob_centers(k, d, seed, device, spread)
    X = torch.empty((hi - lo, d), dtype=dtype, device=device)
    from dalgo.parallel import runtime
    for s in range(0, hi - lo, chunk):
        runtime.heartbeat()   # long generation is progress (stall watchdog)
        e = min(hi - lo, s + chunk)
        u = torch.empty((e - s, 1), dtype=torch.float32, device=device)
        drandom.philox_fill_(u, D=1, row_offset=lo + s, seed=seed, stream=22, a=0.0, b=float(k))
        ids = u.view(-1).long().clamp_(0, k - 1)
        z = torch.empty((e - s, d), dtype=torch.float32, device=device)
        drandom.philox_fill_(z, D=d, row_offset=lo + s, seed=seed, stream=23, dist=drandom.NORMAL,
                             a=0.0, b=noise)
        X[s:e] = (C[ids] + z).to(dtype)
    return X
