"""Checkpoint / resume (absent in the reference).

State is replicated across ranks (models, centres, ranks, factors), so rank 0
writes one file; per-rank state (EASGD local models) is stored by every rank in
its own file. Loading uses ``torch.load(..., weights_only=True)`` only.
"""
from __future__ import annotations

import os

import torch


def path_for(ckpt_dir: str, name: str, rank: int | None = None) -> str:
    fn = f"{name}.pt" if rank is None else f"{name}.rank{rank}.pt"
    return os.path.join(ckpt_dir, fn)


def save(state: dict, ckpt_dir: str, name: str, rank: int = 0, per_rank: bool = False) -> str | None:
    """Collective: every rank calls it (rank 0 writes unless ``per_rank``). A device
    collective that timed out on any rank raises here on every rank, so a poisoned
    state is never written."""
    from dalgo.parallel import comm
    comm.check_device_errors("checkpoint save")
    if not per_rank and rank != 0:
        return None
    os.makedirs(ckpt_dir, exist_ok=True)
    p = path_for(ckpt_dir, name, rank if per_rank else None)
    tmp = p + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, p)   # atomic: a crash never leaves a torn checkpoint
    return p


def load(ckpt_dir: str, name: str, rank: int = 0, per_rank: bool = False) -> dict | None:
    p = path_for(ckpt_dir, name, rank if per_rank else None)
    if not os.path.exists(p):
        return None
    return torch.load(p, map_location="cpu", weights_only=True)
