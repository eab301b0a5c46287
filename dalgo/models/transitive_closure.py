"""Transitive closure (graph_computation/transitive_closure.py).

Reference: paths = edges; repeat  paths <- distinct(paths U {(x,z) : (x,y) in E,
(y,z) in paths})  until count(paths) stops changing (:31-40), printing the final
size as "The original graph has %i paths" (:42; the text is the reference's).

Two engines, both partitioned by the path TARGET z (columns of P are
independent, so ranks need no communication except the int64 count all-reduce):
  * dense  — P^T as a 0/1 uint8 matrix, one fused int8-MFMA boolean-GEMM round
             per iteration (K9, csrc/kernels/closure.hip). Best up to ~100k
             vertices (n^2 bytes per matrix).
  * sparse — semi-naive set iteration on packed int64 (x<<32|z) keys: only last
             round's NEW paths are joined (same fixpoint and per-round counts as the
             reference's naive join). On the GPU every rank keeps its paths as an
             append-only key array plus a device hash set (K9 sparse,
             csrc/kernels/tc_sparse.hip): one kernel expands the frontier through the
             in-edge CSR and inserts each candidate with a 64-bit CAS, so dedup, the
             test against all earlier paths and the merge are one pass with no sort.
             The CPU reference path uses torch sort / unique / isin.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from dalgo.ops import _ext
from dalgo.parallel import comm
from dalgo.utils.obs import NULL_PHASE


@dataclass
class ClosureResult:
    n_paths: int
    counts: list = field(default_factory=list)   # count after each round (incl. initial)


def compact_ids(src: torch.Tensor, dst: torch.Tensor):
    """Relabel vertex ids to 0..n-1 (returns new src, dst, id table)."""
    ids, inv = torch.unique(torch.cat([src, dst]), return_inverse=True)
    n = src.numel()
    return inv[:n], inv[n:], ids


# K9 (csrc/kernels/closure.hip): 256 x 256 tiles (8 waves, 128-B K stages) when the padded
# sizes allow, else 128 x 128. n = 16384, 1 x MI355X: 2.33 POP/s int8 (torch._int_mm, the
# plain library GEMM of the same shape without the OR epilogue: 2.86 POP/s)


def _round_up(a, b):
    return (a + b - 1) // b * b


class _Fixpoint:
    """Shared fixpoint driver (transitive_closure.py:31-40) with resumable state: the
    per-round counts travel with the path set in ``state_dict`` (checkpoint/resume,
    SURVEY §5), so a resumed run continues the same trajectory."""
    counts: list
    timer = None   # dalgo.utils.obs.PhaseTimer (None = off)

    def _ph(self, name: str):
        return self.timer.phase(name) if self.timer is not None else NULL_PHASE

    def _initial_count(self) -> int:
        raise NotImplementedError

    def run(self, max_rounds: int = 1 << 30, callback=None) -> ClosureResult:
        if not self.counts:
            self.counts = [self._initial_count()]
        cnt = self.counts[-1]
        done = len(self.counts) > 1 and self.counts[-1] == self.counts[-2]
        rounds = 0
        while not done and rounds < max_rounds:
            with self._ph("round"):
                nxt = self.step()
            self.counts.append(nxt)
            rounds += 1
            done = nxt == cnt
            cnt = nxt
            if callback is not None:
                callback(self)
        return ClosureResult(cnt, list(self.counts))

    @property
    def converged(self) -> bool:
        return len(self.counts) > 1 and self.counts[-1] == self.counts[-2]


class DenseClosure(_Fixpoint):
    def __init__(self, src: torch.Tensor, dst: torch.Tensor, n: int, rank: int = 0, world: int = 1,
                 device="cpu"):
        dev = torch.device(device)
        self.dev = dev
        self.n = n
        # 256 x 256 K9 tiles once the graph is big enough to fill them, 128 x 128 below
        al = 256 if n > 128 else 128
        self.npad = _round_up(max(n, 1), al)
        sl = _round_up((self.npad + world - 1) // world, al)
        self.z_lo = min(self.npad, rank * sl)
        self.z_hi = min(self.npad, (rank + 1) * sl)
        self.nz = sl
        dt = torch.uint8 if dev.type == "cuda" else torch.float32
        src = src.to(dev).long()
        dst = dst.to(dev).long()
        self.A = torch.zeros((self.npad, self.npad), dtype=dt, device=dev)
        self.A[src, dst] = 1
        self.T = torch.zeros((self.nz, self.npad), dtype=dt, device=dev)
        m = (dst >= self.z_lo) & (dst < self.z_hi)
        self.T[dst[m] - self.z_lo, src[m]] = 1            # T[z][x] = P[x][z]
        self.T2 = torch.zeros_like(self.T)
        self.count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.counts: list = []

    def nnz(self) -> int:
        c = (self.T != 0).sum().reshape(1).to(torch.int64)
        return comm.all_reduce_count(c)

    def step(self) -> int:
        if self.dev.type == "cuda":
            self.count.zero_()
            _ext.ops().tc_step(self.A, self.T, self.T2, self.count)
        else:
            C = self.T @ self.A.T                           # C^T[z][x] = sum_y T[z][y] A[x][y]
            self.T2.copy_(((self.T != 0) | (C > 0.5)).to(self.T.dtype))
            self.count.copy_((self.T2 != 0).sum().reshape(1))
        self.T, self.T2 = self.T2, self.T
        return comm.all_reduce_count(self.count)

    def _initial_count(self) -> int:
        return self.nnz()

    def state_dict(self) -> dict:
        """This rank's slice of P^T, bit-packed (n^2 / 8 bytes for the whole graph)."""
        bits = np.packbits((self.T != 0).cpu().numpy(), axis=1)
        return {"engine": "dense", "n": self.n, "z_lo": self.z_lo, "z_hi": self.z_hi,
                "nz": self.nz, "npad": self.npad, "T_bits": torch.from_numpy(bits),
                "counts": torch.tensor(self.counts, dtype=torch.int64)}

    def load_state_dict(self, sd: dict):
        if sd.get("engine") != "dense" or (sd["n"], sd["z_lo"], sd["z_hi"], sd["npad"]) != \
                (self.n, self.z_lo, self.z_hi, self.npad):
            raise ValueError("checkpoint is for a different graph or rank partition")
        t = np.unpackbits(sd["T_bits"].numpy(), axis=1, count=self.npad)
        self.T.copy_(torch.from_numpy(t).to(self.T.dtype))
        self.counts = [int(c) for c in sd["counts"].tolist()]


class SparseClosure(_Fixpoint):
    """Semi-naive closure over path keys (x << 32 | z) of this rank's targets
    (z % world == rank); the edges are replicated as an in-edge CSR (in_ptr / in_src,
    the reversed edge RDD of transitive_closure.py:27).

    GPU (K9 sparse, csrc/kernels/tc_sparse.hip): the path set is an append-only key
    array plus a device hash set; a round expands only the last round's new paths
    (the frontier) through the in-edges and inserts every candidate with one 64-bit
    CAS -- dedup, the test against earlier paths and the merge into P in one kernel,
    no sort. CPU: the torch reference (repeat_interleave join, unique, isin, sort).
    """

    def __init__(self, src: torch.Tensor, dst: torch.Tensor, rank: int = 0, world: int = 1,
                 n: int | None = None, device="cpu"):
        dev = torch.device(device)
        src = src.to(dev).long()
        dst = dst.to(dev).long()
        self.dev = dev
        n = int(max(src.max().item(), dst.max().item()) + 1) if n is None else n
        if n >= 1 << 31:
            raise ValueError("sparse closure: vertex ids must fit in 31 bits")
        self.n = n
        # edges grouped by their TARGET y: in_ptr / in_src (the reversed edge RDD)
        order = torch.argsort(dst * n + src)
        ys, xs = dst[order], src[order]
        self.in_src = xs
        self.in_ptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        self.in_ptr[1:] = torch.cumsum(torch.bincount(ys, minlength=n), 0)
        self.rank, self.world = rank, world
        self.counts: list = []
        own = (dst % world) == rank
        init = (src[own] << 32) | dst[own]
        self.gpu = dev.type == "cuda"
        if self.gpu:
            from dalgo.ops import _ext
            self._ops = _ext.ops()
            self.in_src32 = xs.to(torch.int32).contiguous()
            self.n_keys_dev = torch.zeros(1, dtype=torch.int64, device=dev)
            self.err = torch.zeros(1, dtype=torch.int32, device=dev)
            self._alloc(max(1024, 4 * init.numel()))
            self._ops.tcs_insert(init.contiguous(), self.table, True, self.keys, self.n_keys_dev,
                                 self.err)
            self.n_keys = int(self.n_keys_dev.item())
            self.d0 = 0                      # frontier = keys[d0 : n_keys]
            self.rounds_candidates: list = []
        else:
            self.P = torch.unique(init)
            self.delta = self.P

    # ------------------------------------------------------------------ GPU engine
    def _alloc(self, want_keys: int):
        """Table of the next power of two >= 2 x want_keys slots; key array of half that."""
        size = 1 << max(10, (2 * int(want_keys) - 1).bit_length())
        self.table = torch.full((size,), -1, dtype=torch.int64, device=self.dev)
        keys = torch.empty(size // 2, dtype=torch.int64, device=self.dev)
        if getattr(self, "keys", None) is not None and self.n_keys:
            keys[: self.n_keys].copy_(self.keys[: self.n_keys])
        self.keys = keys

    def _grow(self, want_keys: int):
        self._alloc(want_keys)
        if self.n_keys:
            # rehash the existing paths (no append: they are already in `keys`)
            self._ops.tcs_insert(self.keys[: self.n_keys], self.table, False, self.keys,
                                 self.n_keys_dev, self.err)

    def _gpu_step(self) -> int:
        d0, d1 = self.d0, self.n_keys
        nd = d1 - d0
        if nd:
            with self._ph("degrees"):
                excl = torch.zeros(nd + 1, dtype=torch.int64, device=self.dev)
                self._ops.tcs_degree(self.keys, d0, nd, self.in_ptr, excl[1:])
                torch.cumsum(excl[1:], 0, out=excl[1:])
            total = int(excl[nd].item())
            self.rounds_candidates.append(total)
            c = 0
            while c < total:
                free = self.table.numel() // 2 - self.n_keys
                if free < min(total - c, self.table.numel() // 8):
                    # more room first: the chunk below can add at most its candidate count
                    self._grow(2 * (self.n_keys + min(total - c, self.n_keys + 1)))
                    continue
                m = min(total - c, free)
                with self._ph("expand+insert"):
                    self._ops.tcs_expand(self.keys, d0, nd, excl, c, c + m, self.in_ptr,
                                         self.in_src32, self.table, self.n_keys_dev, self.err)
                self.n_keys = int(self.n_keys_dev.item())
                c += m
            if int(self.err.item()):
                raise RuntimeError("sparse closure: hash-set capacity invariant broken")
        self.d0 = d1
        return comm.all_reduce_count(self.n_keys, device=self.dev)

    # ------------------------------------------------------------------ CPU engine
    def _join(self, delta: torch.Tensor) -> torch.Tensor:
        y = delta >> 32
        z = delta & 0xFFFFFFFF
        deg = self.in_ptr[y + 1] - self.in_ptr[y]
        tot = int(deg.sum().item())
        if tot == 0:
            return delta[:0]
        rep = torch.repeat_interleave(torch.arange(delta.numel(), device=self.dev), deg)
        start = torch.repeat_interleave(self.in_ptr[y], deg)
        within = torch.arange(tot, device=self.dev) - torch.repeat_interleave(
            torch.cumsum(deg, 0) - deg, deg)
        x = self.in_src[start + within]
        return torch.unique((x << 32) | z[rep])

    def step(self) -> int:
        if self.gpu:
            return self._gpu_step()
        new = self._join(self.delta)
        if new.numel():
            new = new[~torch.isin(new, self.P)]
        self.P = torch.sort(torch.cat([self.P, new])).values
        self.delta = new
        return comm.all_reduce_count(self.P.numel(), device=self.dev)

    def _initial_count(self) -> int:
        n = self.n_keys if self.gpu else self.P.numel()
        return comm.all_reduce_count(n, device=self.dev)

    def paths(self) -> torch.Tensor:
        """This rank's path keys (x << 32 | z), sorted."""
        if self.gpu:
            return torch.sort(self.keys[: self.n_keys]).values
        return self.P

    def frontier(self) -> torch.Tensor:
        if self.gpu:
            return torch.sort(self.keys[self.d0: self.n_keys]).values
        return self.delta

    def state_dict(self) -> dict:
        """This rank's path set and last round's new paths (semi-naive frontier)."""
        return {"engine": "sparse", "n": self.n, "rank": self.rank, "world": self.world,
                "P": self.paths().cpu(), "delta": self.frontier().cpu(),
                "counts": torch.tensor(self.counts, dtype=torch.int64)}

    def load_state_dict(self, sd: dict):
        if sd.get("engine") != "sparse" or (sd["n"], sd["rank"], sd["world"]) != \
                (self.n, self.rank, self.world):
            raise ValueError("checkpoint is for a different graph or rank partition")
        P = sd["P"].to(self.dev)
        delta = sd["delta"].to(self.dev)
        self.counts = [int(c) for c in sd["counts"].tolist()]
        if not self.gpu:
            self.P, self.delta = P, delta
            return
        # key array = (P \ delta) followed by delta, so the frontier is the contiguous tail
        old = P[~torch.isin(P, delta)] if delta.numel() else P
        self.keys = None
        self.n_keys = 0
        self._alloc(max(1024, 2 * P.numel()))
        self.n_keys_dev.zero_()
        self._ops.tcs_insert(old.contiguous(), self.table, True, self.keys, self.n_keys_dev,
                             self.err)
        d0 = int(self.n_keys_dev.item())
        self._ops.tcs_insert(delta.contiguous(), self.table, True, self.keys, self.n_keys_dev,
                             self.err)
        self.n_keys = int(self.n_keys_dev.item())
        self.d0 = d0
        if self.n_keys != P.numel():
            raise ValueError("sparse closure checkpoint: path set is not duplicate-free")
