"""Graph ops: R-MAT generation, destination-partitioned edge lists, PageRank K4.

GPU tensors run csrc/kernels/pagerank.hip; CPU tensors run the torch references.
A rank's graph shard is its destination vertex range [v_lo, v_hi) and exactly the
in-edges of those vertices, sorted by (dst, src) and deduplicated — the
``links.distinct().groupByKey()`` of graph_computation/pagerank.py:41 done once,
on device, as a sort + unique (no per-iteration shuffles).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from dalgo.ops import _ext
from dalgo.utils import philox


# ------------------------------------------------------------------ generation
def rmat_edges(n_edges: int, scale: int, *, seed: int = 1, e_off: int = 0, a=0.57, b=0.19,
               c=0.19, scramble: bool = True, device="cpu"):
    """Edges [e_off, e_off+n) of the deterministic R-MAT stream (Graph500 a,b,c,d)."""
    device = torch.device(device)
    src = torch.empty(n_edges, dtype=torch.int32, device=device)
    dst = torch.empty(n_edges, dtype=torch.int32, device=device)
    if device.type == "cuda":
        _ext.ops().rmat_edges(int(seed), int(scale), int(e_off), float(a), float(b), float(c),
                              bool(scramble), src, dst)
        return src, dst
    s, d = _rmat_cpu(n_edges, scale, seed, e_off, a, b, c, scramble)
    src.copy_(torch.from_numpy(s))
    dst.copy_(torch.from_numpy(d))
    return src, dst


def _scramble_np(v, scale, k0, k1):
    mask = np.uint64((1 << scale) - 1)
    v = v.astype(np.uint64)
    v = (v * np.uint64(k0 | 1)) & np.uint64(0xFFFFFFFF) & mask
    v ^= v >> np.uint64(scale // 2 + 1)
    v = (v * np.uint64(k1 | 1)) & np.uint64(0xFFFFFFFF) & mask
    v ^= v >> np.uint64(scale // 3 + 1)
    v = (v * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF) & mask
    return v


def _rmat_cpu(n, scale, seed, e_off, a, b, c, scramble):
    pa = int(a * 256 + 0.5)
    pab = int((a + b) * 256 + 0.5)
    pabc = int((a + b + c) * 256 + 0.5)
    e = np.arange(e_off, e_off + n, dtype=np.uint64)
    words = []
    for half in (0, 1):
        blk = np.uint64(2) * e + np.uint64(half)
        c0 = (blk & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        c1 = (blk >> np.uint64(32)).astype(np.uint32)
        c2 = np.full(n, 7, dtype=np.uint32)
        c3 = np.zeros(n, dtype=np.uint32)
        words.extend(philox.philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    s = np.zeros(n, dtype=np.uint64)
    d = np.zeros(n, dtype=np.uint64)
    for lvl in range(scale):
        u = (words[lvl >> 2] >> np.uint32(8 * (lvl & 3))) & np.uint32(0xFF)
        sb = (u >= pab).astype(np.uint64)
        db = ((u >= pabc) | ((u >= pa) & (u < pab))).astype(np.uint64)
        s = (s << np.uint64(1)) | sb
        d = (d << np.uint64(1)) | db
    if scramble:
        k0 = (seed & 0xFFFFFFFF) ^ 0x5BD1E995
        k1 = ((seed >> 32) & 0xFFFFFFFF) ^ 0x27D4EB2F
        s = _scramble_np(s, scale, k0, k1)
        d = _scramble_np(d, scale, k0, k1)
    return s.astype(np.int32), d.astype(np.int32)


# ------------------------------------------------------------------ shards
@dataclass
class GraphShard:
    src: torch.Tensor      # int32 [E_pad], global source ids (-1 padding)
    dstl: torch.Tensor     # int32 [E_pad], LOCAL destination ids (-1 padding)
    n_edges: int           # real local edges
    v_lo: int
    v_hi: int
    n_vertices: int        # global vertex-id space size
    slice_size: int        # vertices per rank slice (padded, for all_gather)
    new_id: torch.Tensor | None = None   # old -> new vertex id (degree reordering), if any

    @property
    def n_local(self) -> int:
        return self.v_hi - self.v_lo


def vertex_slices(n_vertices: int, world: int) -> int:
    return (n_vertices + world - 1) // world


def build_shard(src: torch.Tensor, dst: torch.Tensor, n_vertices: int, rank: int, world: int,
                dedup: bool = True) -> GraphShard:
    """Keep the edges whose destination this rank owns; sort by (dst, src), dedup, pad."""
    sl = vertex_slices(n_vertices, world)
    v_lo, v_hi = rank * sl, min(n_vertices, (rank + 1) * sl)
    m = (dst >= v_lo) & (dst < v_hi)
    s = src[m].to(torch.int64)
    d = dst[m].to(torch.int64) - v_lo
    key = (d << 32) | s
    key = torch.unique(key) if dedup else torch.sort(key).values
    return _shard_from_keys(key, v_lo, v_hi, n_vertices, sl)


def _shard_from_keys(key, v_lo, v_hi, n_vertices, sl) -> GraphShard:
    E = int(key.numel())
    Ep = ((E + 3) // 4) * 4
    src = torch.full((Ep,), -1, dtype=torch.int32, device=key.device)
    dstl = torch.full((Ep,), -1, dtype=torch.int32, device=key.device)
    src[:E] = (key & 0xFFFFFFFF).to(torch.int32)
    dstl[:E] = (key >> 32).to(torch.int32)
    return GraphShard(src, dstl, E, v_lo, v_hi, n_vertices, sl)


def merge_shards(parts: list, v_lo, v_hi, n_vertices, sl, dedup=True) -> GraphShard:
    """Combine chunk-wise filtered (src, dstl) parts (streamed generation)."""
    keys = torch.cat([(d.to(torch.int64) << 32) | s.to(torch.int64) for s, d in parts])
    keys = torch.unique(keys) if dedup else torch.sort(keys).values
    return _shard_from_keys(keys, v_lo, v_hi, n_vertices, sl)


def local_outdeg(shard: GraphShard) -> torch.Tensor:
    """Out-degree contribution of this shard's edges (sum over ranks = global out-degree)."""
    s = shard.src[: shard.n_edges].to(torch.int64)
    return torch.bincount(s, minlength=shard.n_vertices).to(torch.int32)


# ------------------------------------------------------------------ K4 kernels
def pr_spmv(shard: GraphShard, c_full: torch.Tensor, acc: torch.Tensor, pres: torch.Tensor):
    """acc[v] = sum_{u->v, c[u] >= 0} c[u];  pres[v] = any such edge  (acc/pres zeroed by caller)."""
    if c_full.is_cuda:
        _ext.ops().pr_spmv(shard.src, shard.dstl, c_full, acc, pres)
        return
    E = shard.n_edges
    s = shard.src[:E].long()
    d = shard.dstl[:E].long()
    cv = c_full[s]
    acc.index_add_(0, d, cv.clamp_min(0))
    hit = torch.zeros_like(pres)
    hit.index_add_(0, d, (cv >= 0).to(pres.dtype))
    pres.copy_((hit > 0).to(pres.dtype))


def pr_update(acc, pres, outdeg_local, q, invN, mode, r, c, dangling_in=None, dangling_out=None):
    if acc.is_cuda:
        _ext.ops().pr_update(acc, pres, outdeg_local, float(q), float(invN), int(mode),
                             dangling_in, r, c, dangling_out)
        return
    od = outdeg_local.to(acc.dtype)
    if mode == 0:
        p = pres != 0
        rv = torch.where(p, q * invN + (1 - q) * acc, torch.full_like(acc, -1.0))
        r.copy_(rv)
        c.copy_(torch.where(p & (od > 0), rv / od.clamp_min(1), torch.full_like(acc, -1.0)))
    else:
        dang = float(dangling_in.reshape(-1)[0]) if dangling_in is not None else 0.0
        rv = q * invN + (1 - q) * (acc + dang * invN)
        r.copy_(rv)
        c.copy_(torch.where(od > 0, rv / od.clamp_min(1), torch.zeros_like(acc)))
        if dangling_out is not None:
            dangling_out += torch.where(od == 0, rv, torch.zeros_like(rv)).sum()
