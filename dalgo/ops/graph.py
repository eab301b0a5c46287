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


# ------------------------------------------------------------------ propagation blocking
@dataclass
class BlockedLayout:
    """Edge layout of the propagation-blocked SpMV (pb_spmv): see csrc/kernels/pagerank.hip.

    psrc/ppos: phase-1 edge list (global src id, slot in the binned array) in
    tile order: tiles of ``tile`` consecutive edges in SOURCE order, each tile
    re-sorted by slot, so the c[src] reads of a tile stay inside a narrow source
    range while its writes form contiguous runs per bin (coalesced stores).
    val/dloc: the destination-binned array (value written per iteration, static
    destination offset inside the bin; slots of a bin are in source order).
    chunks: contiguous slot ranges of one bin; a bin longer than ``chunk`` slots
    is split, its chunks write partial slabs that pb_combine sums in order."""
    psrc: torch.Tensor
    ppos: torch.Tensor
    val: torch.Tensor
    dloc: torch.Tensor
    chunk_lo4: torch.Tensor
    chunk_bin: torch.Tensor
    chunk_slab: torch.Tensor
    slab: torch.Tensor
    split_bin: torch.Tensor
    split_first: torch.Tensor
    split_count: torch.Tensor
    bin_width: int
    n_local: int


def build_blocked(shard: GraphShard, bin_width: int = 16384, chunk: int = 1 << 18,
                  tile: int = 1 << 16) -> BlockedLayout:
    """One-time construction from a (dst, src)-sorted shard (device sorts)."""
    if bin_width not in (8192, 16384):
        raise ValueError("bin_width must be 8192 or 16384 (LDS accumulator sizes of the kernel)")
    dev = shard.src.device
    E = shard.n_edges
    s = shard.src[:E].to(torch.int64)
    d = shard.dstl[:E].to(torch.int64)
    nl = shard.n_local
    nbins = max(1, (nl + bin_width - 1) // bin_width)
    b = d // bin_width
    # slots: bins in order, inside a bin edges in source order, each bin padded to 4
    order2 = torch.argsort(b * (shard.n_vertices + 1) + s, stable=True)
    inv2 = torch.empty_like(order2)
    inv2[order2] = torch.arange(E, device=dev)
    del order2
    cnt = torch.bincount(b, minlength=nbins)
    start_u = torch.cumsum(cnt, 0) - cnt
    cntp = (cnt + 3) // 4 * 4
    start_p = torch.cumsum(cntp, 0) - cntp
    Ep = max(int(cntp.sum().item()) if E else 0, 4)
    pos = start_p[b] + (inv2 - start_u[b])
    del inv2
    val = torch.full((Ep,), -1.0, dtype=torch.float32, device=dev)
    dloc = torch.zeros(Ep, dtype=torch.int16, device=dev)
    dl = d - b * bin_width
    dloc[pos] = dl.to(torch.int32).to(torch.int16)        # < 16384: fits int16 as is
    # phase-1 order: source order, then slot order inside each tile
    order1 = torch.argsort(s, stable=True)
    pos1 = pos[order1]
    t_id = torch.arange(E, device=dev) // max(1, tile)
    order_t = torch.argsort(t_id * Ep + pos1)
    E4 = (E + 3) // 4 * 4
    psrc = torch.full((max(E4, 4),), -1, dtype=torch.int32, device=dev)
    ppos = torch.zeros(max(E4, 4), dtype=torch.int32, device=dev)
    psrc[:E] = s[order1][order_t].to(torch.int32)
    ppos[:E] = pos1[order_t].to(torch.int32)
    del order1, pos1, t_id, order_t
    # chunks (host): split each non-empty bin into <= chunk-slot pieces (multiples of 4)
    cntp_h = cntp.cpu().tolist()
    start_h = start_p.cpu().tolist()
    chunk = max(4, chunk // 4 * 4)
    lo4, bins, slab_of, sp_bin, sp_first, sp_cnt = [], [], [], [], [], []
    nslab = 0
    for bi, (st, n) in enumerate(zip(start_h, cntp_h)):
        if n == 0:
            continue
        pieces = list(range(st, st + n, chunk))
        if len(pieces) > 1:
            sp_bin.append(bi)
            sp_first.append(nslab)
            sp_cnt.append(len(pieces))
        for p0 in pieces:
            lo4.append(p0 // 4)
            bins.append(bi)
            if len(pieces) > 1:
                slab_of.append(nslab)
                nslab += 1
            else:
                slab_of.append(-1)
    lo4.append(Ep // 4 if E else 0)
    # the invariants the kernels rely on (checked once, here)
    assert E == 0 or (int(pos.max()) < Ep and int(dl.max()) < bin_width and int(dl.min()) >= 0)
    assert E == 0 or (int(s.min()) >= 0 and int(s.max()) < shard.n_vertices)
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device=dev)
    return BlockedLayout(psrc, ppos, val, dloc,
                         torch.tensor(lo4, dtype=torch.int64, device=dev), i32(bins), i32(slab_of),
                         torch.zeros(max(nslab, 1) * bin_width, dtype=torch.float32, device=dev),
                         i32(sp_bin), i32(sp_first), i32(sp_cnt), bin_width, nl)


def pb_spmv(lay: BlockedLayout, c_full: torch.Tensor, acc: torch.Tensor, pres: torch.Tensor):
    """Same result as :func:`pr_spmv` (acc/pres zeroed by the caller)."""
    if c_full.is_cuda:
        _ext.ops().pb_spmv(lay.psrc, lay.ppos, c_full, lay.val, lay.dloc, lay.chunk_lo4,
                           lay.chunk_bin, lay.chunk_slab, lay.bin_width, acc, pres, lay.slab,
                           lay.split_bin, lay.split_first, lay.split_count)
        return
    # CPU reference of the two phases
    m = lay.psrc >= 0
    lay.val[lay.ppos[m].long()] = c_full[lay.psrc[m].long()]
    lo = lay.chunk_lo4.tolist()
    for k, bi in enumerate(lay.chunk_bin.tolist()):
        v = lay.val[lo[k] * 4: lo[k + 1] * 4]
        dd = lay.dloc[lo[k] * 4: lo[k + 1] * 4].long() + bi * lay.bin_width
        keep = v >= 0
        acc.index_add_(0, dd[keep], v[keep])
        pres[dd[keep]] = 1


# ------------------------------------------------------------------ K4 kernels
def pr_spmv(shard: GraphShard, c_full: torch.Tensor, acc: torch.Tensor, pres: torch.Tensor,
            accumulate: bool = False):
    """acc[v] = sum_{u->v, c[u] >= 0} c[u];  pres[v] = any such edge  (acc/pres zeroed by caller).
    ``accumulate``: a further pass over another edge subset of the same rows (adds to acc,
    ORs pres)."""
    if c_full.is_cuda:
        _ext.ops().pr_spmv(shard.src, shard.dstl, c_full, acc, pres, bool(accumulate))
        return
    E = shard.n_edges
    s = shard.src[:E].long()
    d = shard.dstl[:E].long()
    cv = c_full[s]
    acc.index_add_(0, d, cv.clamp_min(0))
    hit = torch.zeros_like(pres)
    hit.index_add_(0, d, (cv >= 0).to(pres.dtype))
    if accumulate:
        hit += pres
    pres.copy_((hit > 0).to(pres.dtype))


# ------------------------------------------------------------------ XCD-partitioned K4
XCD_PARTS = 8


@dataclass
class XcdLayout:
    """Edges split into 8 source-line parts for pr_spmv_xcd (csrc/kernels/pagerank.hip):
    part p holds the edges whose source's 128-B contribution line was assigned to p,
    each part sorted by (dst, src) and padded to whole 256-edge windows; part p is swept
    by the blocks with blockIdx % 8 == p (one XCD), so each XCD's L2 caches only its
    own lines. Lines are dealt to parts by descending edge count in snake order
    (0..7, 7..0, ...), which balances the parts' edge counts."""
    src: torch.Tensor        # int32 [E_pad]
    dstl: torch.Tensor       # int32 [E_pad]
    base: torch.Tensor       # int64 [9] part offsets (device)
    counts: list             # real edges per part
    e_max: int               # largest padded part
    n_local: int
    acc: torch.Tensor        # f32 [8, n_local]: per-part sums, -0.0 = no record


def build_xcd(shard: GraphShard) -> XcdLayout:
    E = shard.n_edges
    dev = shard.src.device
    s = shard.src[:E]
    d = shard.dstl[:E]
    line = (s >> 5).to(torch.int64)
    n_lines = int(line.max().item()) + 1 if E else 1
    cnt = torch.bincount(line, minlength=n_lines)
    order = torch.argsort(cnt, descending=True, stable=True)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(n_lines, device=dev)
    r = rank % (2 * XCD_PARTS)
    part_of_line = torch.where(r < XCD_PARTS, r, 2 * XCD_PARTS - 1 - r)
    part = part_of_line[line]
    perm = torch.argsort(part, stable=True)          # keeps the (dst, src) order per part
    counts = torch.bincount(part, minlength=XCD_PARTS).tolist()
    padded = [((c + 255) // 256) * 256 for c in counts]
    tot = sum(padded)
    src = torch.full((max(tot, 4),), -1, dtype=torch.int32, device=dev)
    dstl = torch.full((max(tot, 4),), -1, dtype=torch.int32, device=dev)
    base, off, o2 = [0], 0, 0
    ps, pd = s[perm], d[perm]
    for c, p in zip(counts, padded):
        src[off: off + c] = ps[o2: o2 + c]
        dstl[off: off + c] = pd[o2: o2 + c]
        off += p
        o2 += c
        base.append(off)
    nl = shard.n_local
    acc = torch.full((XCD_PARTS, max(nl, 1)), -0.0, dtype=torch.float32, device=dev)
    return XcdLayout(src, dstl, torch.tensor(base, dtype=torch.int64, device=dev), counts,
                     max(padded), nl, acc)


def pr_spmv_xcd(xl: XcdLayout, c_full: torch.Tensor):
    """Per-part partial sums of the pull SpMV into xl.acc (see XcdLayout)."""
    _ext.ops().pr_spmv_xcd(xl.src, xl.dstl, xl.base, int(xl.e_max), c_full, xl.acc)


def pr_update_xcd(xl: XcdLayout, outdeg_local, q, invN, mode, r, c, dangling_in=None,
                  dangling_out=None):
    """pr_update over the part sums (summed in part order; parts reset to -0.0)."""
    _ext.ops().pr_update_xcd(xl.acc, outdeg_local, float(q), float(invN), int(mode), dangling_in,
                             r, c, dangling_out)


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
