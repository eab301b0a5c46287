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
    from dalgo.parallel import comm, runtime
    comm.check_device_errors("checkpoint save")
    if not per_rank and rank != 0:
        return None
    os.makedirs(ckpt_dir, exist_ok=True)
    p = path_for(ckpt_dir, name, rank if per_rank else None)
    tmp = p + ".tmp"
    runtime.heartbeat()  # a long write is progress, not a stall (runtime.arm_stall_watchdog)
    torch.save(state, tmp)
    os.replace(tmp, p)   # atomic: a crash never leaves a torn checkpoint
    runtime.heartbeat()
    return p


def load(ckpt_dir: str, name: str, rank: int = 0, per_rank: bool = False) -> dict | None:
    p = path_for(ckpt_dir, name, rank if per_rank else None)
    if not os.path.exists(p):
        return None
    return torch.load(p, map_location="cpu", weights_only=True)


def load_consistent(ckpt_dir: str, name: str, rank: int, *, fingerprint: str,
                    progress) -> dict | None:
    """Collective per-rank resume: every rank loads its own file, then all ranks agree.

    Returns the state on every rank when ALL ranks found a file with the expected
    ``fingerprint`` (e.g. a hash of the input graph) at the same ``progress(state)``
    (e.g. the round count); None on every rank when no rank found one; raises on every
    rank otherwise (a crash between two ranks' saves, a missing file on one rank, a
    checkpoint of a different input) -- ranks that resumed from different points
    would enter different numbers of collectives and hang or reach a wrong fixpoint."""
    from dalgo.parallel import comm, runtime
    sd = load(ckpt_dir, name, rank, per_rank=True)
    found = sd is not None
    match = found and sd.get("fingerprint") == fingerprint
    prog = int(progress(sd)) if match else -1
    dev = runtime.get().device if comm._active() and \
        torch.distributed.get_backend() == "nccl" else torch.device("cpu")
    hi = torch.tensor([int(found), int(match), prog], dtype=torch.int64, device=dev)
    lo = -hi.clone()
    comm.all_reduce_max(hi)
    comm.all_reduce_max(lo)
    any_found, all_found = int(hi[0]), -int(lo[0])
    all_match, p_max, p_min = -int(lo[1]), int(hi[2]), -int(lo[2])
    if not any_found:
        return None
    if not (all_found and all_match and p_min == p_max):
        raise RuntimeError(
            f"inconsistent resume of {name!r}: found on all ranks={bool(all_found)}, same input "
            f"on all ranks={bool(all_match)}, progress min/max={p_min}/{p_max}")
    return sd
