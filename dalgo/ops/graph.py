"""Graph ops: R-MAT generation, destination-partitioned edge lists, PageRank K4.

GPU tensors run csrc/kernels/pagerank.hip; CPU tensors run the torch references.
A rank's graph shard is its destination vertex range [v_lo, v_hi) and exactly the
in-edges of those vertices, sorted by (dst, src) and deduplicated — the
``links.distinct().groupByKey()`` of graph_computation/pagerank.py:41 done once,
on device, as a sort + unique (no per-iteration shuffles).
"""
from __future__ import annotations

from dataclasses import dataclass

import math

import numpy as np
import os

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


def degree_count_(deg: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """deg[v] += #occurrences of v in ids. GPU (int32 deg, int32 ids): one u32 atomic per
    id (csrc/kernels/graph_build.hip), not torch's int64 histogram."""
    if deg.is_cuda and deg.dtype == torch.int32 and ids.dtype == torch.int32:
        _ext.ops().gb_degree(ids.contiguous(), deg)
        return deg
    deg += torch.bincount(ids.long(), minlength=deg.numel()).to(deg.dtype)
    return deg


BUCKET_BITS = 13          # ids per degree bucket: 2^13 (graph_build.hip kBktBits)


def partition_edges(edges: list, bits: int):
    """One rank: every (src, dst) edge packed as src << 32 | dst and partitioned on the high
    source bits (2 radix passes at 2^26 ids), plus the raw out-degree of every source
    (ids < 2^bits, bits > BUCKET_BITS): (packed int64 [E], deg int32 [2^bits])."""
    ops = _ext.ops()
    dev = edges[0][0].device
    n = sum(int(s.numel()) for s, _ in edges)
    packed = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    o = 0
    for s, d in edges:
        ops.gb_pack(s, d, packed[o:o + s.numel()])
        o += int(s.numel())
    out = torch.empty_like(packed)
    deg = torch.zeros(1 << bits, dtype=torch.int32, device=dev)
    ops.gb_degree_packed(packed[:n], int(bits), deg, out)
    del packed
    return out[:n], deg


def relabel_partition_dst(packed: torch.Tensor, new_id: torch.Tensor, bits: int) -> torch.Tensor:
    """Source-partitioned packed edges (:func:`partition_edges`): the sources relabelled in
    place (gathers local to each source bucket), then the edges partitioned on the top 8
    destination bits (one radix pass), so the key pass's destination relabeling reads one
    L2-resident slice of new_id per bucket."""
    ops = _ext.ops()
    n = packed.numel()
    ops.gb_relabel_src(packed, new_id, 1)           # bucketed: id slices staged in LDS
    out = torch.empty_like(packed)
    if n:
        # one radix pass over the top 8 destination bits: 2^(bits - 8)-id buckets (1 MB of
        # new_id at scale 26) stay L2-resident while the key pass walks them
        ops.gb_sort(packed, n, int(bits), out, max(0, int(bits) - 8))
    return out


def owner_partition(src: torch.Tensor, dst: torch.Tensor, new_id: torch.Tensor | None, n_vertices: int,
                    world: int) -> tuple[torch.Tensor, list]:
    """The sharded build's shuffle source (graph_computation/pagerank.py:41 groupByKey over
    W ranks): this rank's input edges relabelled through ``new_id`` and grouped by the rank
    that owns the destination (owner = dst' // slice size), packed src << 32 | dst. Returns
    (packed int64 [E], edges per owner). GPU: two passes of graph_build.hip (relabel + count,
    then an owner-major scatter); CPU: torch."""
    sl = vertex_slices(n_vertices, world)
    if src.is_cuda:
        out = torch.empty(src.numel(), dtype=torch.int64, device=src.device)
        nid = new_id.to(torch.int32).contiguous() if new_id is not None else None
        cnt = _ext.ops().gb_owner_partition(src.contiguous(), dst.contiguous(), nid, sl, world, out)
        return out, [int(x) for x in cnt.tolist()]
    s, d = src.long(), dst.long()
    if new_id is not None:
        s, d = new_id.long()[s], new_id.long()[d]
    owner = d // sl
    order = torch.argsort(owner, stable=True)
    packed = ((s << 32) | d)[order]
    cnt = torch.bincount(owner, minlength=world)[:world]
    return packed, [int(x) for x in cnt.tolist()]


def owner_partition_packed(packed: torch.Tensor, new_id: torch.Tensor | None, n_vertices: int,
                           world: int) -> tuple[torch.Tensor, list]:
    """:func:`owner_partition` over edges already packed with RELABELLED sources and grouped
    on their destination bits (:func:`relabel_partition_dst`): only the destinations go
    through ``new_id`` -- from the L2-resident slice of their bucket instead of random
    gathers over the whole table -- then the owner-major grouping. ``packed`` is consumed
    (overwritten on the GPU). Returns (packed int64 [E], edges per owner)."""
    sl = vertex_slices(n_vertices, world)
    if packed.is_cuda:
        out = torch.empty_like(packed)
        nid = new_id.to(torch.int32).contiguous() if new_id is not None else None
        cnt = _ext.ops().gb_owner_partition_packed(packed.contiguous(), nid, sl, world, out)
        return out, [int(x) for x in cnt.tolist()]
    s, d = packed >> 32, packed & 0xFFFFFFFF
    if new_id is not None:
        d = new_id.long()[d]
    owner = d // sl
    order = torch.argsort(owner, stable=True)
    cnt = torch.bincount(owner, minlength=world)[:world]
    return ((s << 32) | d)[order], [int(x) for x in cnt.tolist()]


def unpack_edges(packed: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(src, dst) int32 of packed src << 32 | dst words."""
    return (packed >> 32).to(torch.int32), (packed & 0xFFFFFFFF).to(torch.int32)


def degree_sorted_(deg: torch.Tensor, ids: torch.Tensor, bits: int) -> torch.Tensor:
    """deg[v] += #occurrences of v in ids (GPU int32, ids < 2^bits): the ids partitioned
    on their high bits (2 radix passes at 2^26 ids), then one LDS histogram per bucket of
    8192 ids, instead of one global atomic per id (graph_build.hip)."""
    _ext.ops().gb_degree_sorted(ids.contiguous(), int(bits), deg)
    return deg


def local_outdeg(shard: GraphShard) -> torch.Tensor:
    """Out-degree contribution of this shard's edges (sum over ranks = global out-degree)."""
    s = shard.src[: shard.n_edges].to(torch.int64)
    return torch.bincount(s, minlength=shard.n_vertices).to(torch.int32)


def _work_items(bin_cnt: torch.Tensor, bin_lo: torch.Tensor, nent: int, items: int, min_piece: int):
    """Phase-2 work items: each bin's contiguous bin-major entry range, a hot bin cut into
    ~cap-entry pieces (each with its own slab, combined in order afterwards); an empty
    bin is one empty item (it writes zeros). Computed where the bin counts live (torch,
    on the device for a GPU build: only the item and slab counts come to the host -- a
    first 64 KB device-to-host read of the counts cost 7-17 ms in a fresh process,
    profiles/round5/r5_24, r5_25). Returns (wi_bin, wi_lo + [nent], wi_slab, split_bin,
    split_first, split_count) as int64 tensors and the slab count."""
    cap = max(int(nent // max(items, 1)), min_piece)
    cnt, lo = bin_cnt.to(torch.int64), bin_lo.to(torch.int64)
    dev = cnt.device
    pieces = torch.clamp((cnt + cap - 1) // cap, min=1)
    step = torch.clamp((cnt + pieces - 1) // pieces, min=1)
    ncut = torch.where(cnt == 0, torch.ones_like(cnt), (cnt + step - 1) // step)   # len(range(lo, lo + cnt, step))
    split = pieces > 1
    total, nslab = (int(x) for x in torch.stack([ncut.sum(), torch.where(split, ncut, 0).sum()]).tolist())
    # item j belongs to bin wb[j] (a search over the inclusive item counts: torch's
    # repeat_interleave cost ~2 ms of host time per call here, profiles/round5/r5_27)
    ends = torch.cumsum(ncut, 0)
    j = torch.arange(total, device=dev, dtype=torch.int64)
    wb = torch.searchsorted(ends, j, right=True)
    k = j - (ends - ncut)[wb]
    wl = lo[wb] + k * torch.where(cnt == 0, torch.zeros_like(step), step)[wb]
    in_split = split[wb]
    slab = torch.where(in_split, torch.cumsum(in_split, 0) - 1, torch.full_like(wb, -1))
    sp_bin = torch.nonzero(split).flatten()
    sp_cnt = ncut[split]
    sp_first = torch.cumsum(sp_cnt, 0) - sp_cnt
    wl = torch.cat([wl, torch.full((1,), nent, dtype=torch.int64, device=dev)])
    return (wb, wl, slab, sp_bin, sp_first, sp_cnt), nslab


# ------------------------------------------------------------------ propagation blocking
SRC_SPAN = 8192          # sources per chunk: the LDS table of pb_gather (csrc/kernels/pr_binned.hip)
CELL_CAP = 1 << 30       # largest (block, bin) cell matrix of the native build (4 B x 3 per cell)
PB_DUMMY = 65536         # val / dloc padding after the entries (kPbDummy in pr_binned.hip)
# phase-2 work items of the native build: a bin with more than nent / items entries is cut
# into pieces, each with its own 128 KB u64 slab that pb_combine sums; items = PB_ITEMS /
# sqrt(W) (a rank holds 1/W of the bins). One rank at scale 26 (4096 bins): 2048 -> 346
# split bins, 1.99-2.05 ms per iteration; 1024 -> 1.98-1.99; 768 -> 1.96-1.97; 640 ->
# 1.96-1.97; 512 -> 1.95-2.00 (profiles/round6/r6_80, r6_84). The W = 8 per-rank share
# (512 bins): 2048 -> 0.48 ms, 768 -> 0.39, 384 -> 0.36, 256 -> 0.365, 192 -> 0.35,
# 128 -> 0.37 (r6_86)
PB_ITEMS = int(os.environ.get("DALGO_PB_ITEMS", "768"))


def pb_items(world: int) -> int:
    return max(128, int(round(PB_ITEMS / math.sqrt(max(1, world)))))
# phase-1 work units of the native build: a source chunk is cut every max(32K, E / PB_UNITS)
# edges. Scale 26, one rank, 3 runs each: 2048 -> 1.986-1.990 ms per iteration, 4096 ->
# 1.953-1.967, 8192 -> 2.024-2.027, 16384 -> 2.200-2.208 (profiles/round6/r6_82)
PB_UNITS = int(os.environ.get("DALGO_PB_UNITS", "4096"))
# wave tiles per work unit (tile length = unit edges / PB_TILES, clamped to [1024, tile]):
# 8 -> 1.962-1.972 ms per iteration, 16 -> 1.916-1.968, 24 -> 1.990-1.995, 32 -> 1.993-2.006
# (scale 26, one rank, profiles/round6/r6_83)
PB_TILES = int(os.environ.get("DALGO_PB_TILES", "16"))


@dataclass
class BlockedLayout:
    """Two-level propagation-blocked SpMV layout (K4b, csrc/kernels/pr_binned.hip).

    chunks: contiguous source ranges [slo, slo + ns), ns <= SRC_SPAN, with about
    ``chunk_edges`` edges each. srcl: the edges sorted by (chunk, dst, src), one u16 per
    edge = source offset in its chunk | 0x4000 on the end edge of a run's first entry |
    0x8000 on the end edge of an entry. An entry is one distinct (chunk, dst) pair; a run
    the entries of one (chunk, bin of ``bin_width`` destinations). Entries are stored
    bin-major (val, dloc = destination offset in the bin): entry e (chunk-major index)
    lives at e + run_delta[run of e]. tiles: ~``tile`` edges starting on an entry
    boundary (one wave each); tile_run = the chunk's run starts before the tile.
    work items: contiguous bin-major entry ranges [wi_lo[i], wi_lo[i + 1]) of one bin; a
    bin split into several items writes partial slabs that pb_combine sums in order."""
    srcl: torch.Tensor
    tile_e: torch.Tensor
    tile_ent: torch.Tensor
    tile_run: torch.Tensor
    chunk_tile: torch.Tensor
    wu_tile: torch.Tensor   # work units (one phase-1 workgroup each): tile ranges of one chunk
    wu_chunk: torch.Tensor
    chunk_slo: torch.Tensor
    chunk_ns: torch.Tensor
    chunk_run: torch.Tensor
    run_delta: torch.Tensor
    val: torch.Tensor
    dloc: torch.Tensor
    wi_bin: torch.Tensor
    wi_lo: torch.Tensor
    wi_slab: torch.Tensor
    slab: torch.Tensor
    split_bin: torch.Tensor
    split_first: torch.Tensor
    split_count: torch.Tensor
    bin_width: int
    n_local: int
    n_chunks: int
    n_entries: int
    n_src: int              # c index space the layout reads: c_full.numel() >= n_src
    max_indeg: int          # largest in-degree (fixed-point range of the accumulators)
    max_runs: int           # most non-empty runs in one chunk (phase 1 stages <= 4096 in LDS)
    bound: torch.Tensor = None   # f64[1] device scratch: this call's destination-sum bound
    n_wu_below: int = 0          # work units whose sources are < src_split (build_blocked)
    wu_bounds: tuple = ()        # work units whose sources are < each of src_splits


def build_blocked(shard: GraphShard, bin_width: int = 16384, chunk_edges: int = 1 << 40,
                  tile: int = 16384, items: int = 2048, min_piece: int = 1 << 14,
                  src_split: int | None = None, src_splits=None) -> BlockedLayout:
    """One-time construction (device sorts) from any shard (src in the c index space).

    chunk_edges: cut a source chunk after ~this many edges. The default (no cut: chunks are
    the SRC_SPAN source blocks) combines the most records per entry (0.44 entries per edge
    at R-MAT scale 26 vs 0.68 at 1M-edge chunks); load balance comes from the work units.
    src_split: no chunk straddles this source index, and ``n_wu_below`` counts the work
    units of the sources below it (the own slice of the ghost index space: their phase 1
    can run while the ghost contributions are still being exchanged).
    src_splits: ascending source indices no chunk straddles (the own slice's end and the
    start of every peer's ghost block); ``wu_bounds[i]`` counts the work units of the
    sources below src_splits[i], so each peer's ghost chunks are one unit range."""
    splits = sorted({int(x) for x in (src_splits or [])} |
                    ({int(src_split)} if src_split is not None else set()))
    if bin_width not in (8192, 16384):
        raise ValueError("bin_width must be 8192 or 16384 (u64 LDS accumulator sizes of the kernel)")
    dev = shard.src.device
    E = shard.n_edges
    nl = shard.n_local
    S = SRC_SPAN
    i32 = lambda x: x.to(torch.int32).contiguous()
    i64 = lambda x: x.to(torch.int64).contiguous()
    it = lambda x: torch.tensor(x, dtype=torch.int32, device=dev)
    nbins = max(1, (nl + bin_width - 1) // bin_width)
    if E == 0:        # no chunks; one empty work item per bin still writes every output
        z = torch.zeros(1, dtype=torch.int32, device=dev)
        nb0 = (nl + bin_width - 1) // bin_width
        return BlockedLayout(torch.zeros(16, dtype=torch.int16, device=dev),
                             torch.zeros(1, dtype=torch.int64, device=dev), z[:0], z[:0], z.clone(),
                             z.clone(), z[:0], z[:0], z[:0], z.clone(), z[:0],
                             torch.zeros(PB_DUMMY, device=dev),
                             torch.zeros(PB_DUMMY, dtype=torch.int16, device=dev),
                             torch.arange(nb0, dtype=torch.int32, device=dev),
                             torch.zeros(nb0 + 1, dtype=torch.int64, device=dev),
                             torch.full((nb0,), -1, dtype=torch.int32, device=dev),
                             torch.zeros(1, dtype=torch.int64, device=dev), z[:0], z[:0], z[:0],
                             bin_width, nl, 0, 0, 0, 0, 0,
                             torch.zeros(1, dtype=torch.float64, device=dev))
    s = shard.src[:E].to(torch.int64)
    d = shard.dstl[:E].to(torch.int64)
    n_src = int(s.max().item()) + 1
    max_indeg = int(torch.bincount(d, minlength=nl).max().item())
    assert int(s.min().item()) >= 0 and int(d.min().item()) >= 0 and int(d.max().item()) < nl
    # chunks: source blocks of S ids, cut further every ~chunk_edges edges (on source
    # boundaries); only sources with edges define chunks
    outd = torch.bincount(s, minlength=n_src)
    cs = torch.cumsum(outd, 0) - outd
    ids = torch.arange(n_src, device=dev)
    if splits:                    # source blocks restart at every split: no straddling chunk
        bnd = torch.tensor([0] + splits, dtype=torch.int64, device=dev)
        seg = torch.searchsorted(bnd, ids, right=True) - 1
        seg_len = torch.diff(torch.cat([bnd, torch.tensor([max(n_src, splits[-1])], device=dev)]))
        nblk = (seg_len + S - 1) // S
        base = torch.cumsum(nblk, 0) - nblk
        blk = base[seg] + (ids - bnd[seg]) // S
        del bnd, seg, seg_len, nblk, base
    else:
        blk = ids // S
    key = blk * (E // chunk_edges + 2) + cs // chunk_edges
    del ids, blk
    has = torch.nonzero(outd > 0).flatten()
    kh = key[has]
    new = torch.ones_like(kh, dtype=torch.bool)
    new[1:] = kh[1:] != kh[:-1]
    cid = torch.cumsum(new.to(torch.int64), 0) - 1
    nch = int(cid[-1].item()) + 1
    slo = has[new]
    last = torch.ones_like(new)
    last[:-1] = new[1:]
    ns = has[last] - slo + 1
    assert int(ns.max().item()) <= S
    cid_src = torch.full((n_src,), -1, dtype=torch.int64, device=dev)
    cid_src[has] = cid
    del outd, cs, key, has, kh, new, last, cid
    ec = cid_src[s]
    del cid_src
    assert nch * nl * S < (1 << 62)
    k = (ec * nl + d) * S + (s - slo[ec])
    del ec, s, d
    k = torch.sort(k).values
    ek = k // S                                       # entry key = chunk * nl + dst
    sl = k - ek * S
    del k
    end = torch.ones(E, dtype=torch.bool, device=dev)
    end[:-1] = ek[1:] != ek[:-1]
    ent_key = ek[end]
    del ek
    nent = int(ent_key.numel())
    assert nent < (1 << 31) - 8
    end_edge = torch.nonzero(end).flatten()          # end edge of each entry
    e_start = torch.zeros(nent, dtype=torch.int64, device=dev)
    e_start[1:] = end_edge[:-1] + 1
    ent_dst = ent_key % nl
    ent_chunk = ent_key // nl
    ent_bin = ent_dst // bin_width
    # runs: (chunk, bin) groups of consecutive entries (chunk-major order)
    rk = ent_chunk * nbins + ent_bin
    rstart = torch.ones(nent, dtype=torch.bool, device=dev)
    rstart[1:] = rk[1:] != rk[:-1]
    run_first = torch.nonzero(rstart).flatten()      # chunk-major entry index of each run
    run_of_ent = torch.cumsum(rstart.to(torch.int64), 0) - 1
    run_chunk = ent_chunk[run_first]
    run_bin = ent_bin[run_first]
    run_len = torch.diff(torch.cat([run_first, torch.tensor([nent], device=dev)]))
    # bin-major position of each run: bins in order, chunks in order inside a bin
    border = torch.argsort(run_bin * (nch + 1) + run_chunk)
    bm_start = torch.empty_like(run_first)
    bm_start[border] = torch.cumsum(run_len[border], 0) - run_len[border]
    run_delta = bm_start - run_first
    chunk_run = torch.searchsorted(run_chunk, torch.arange(nch + 1, device=dev))
    bin_cnt = torch.bincount(ent_bin, minlength=nbins)

    bin_lo = torch.cumsum(bin_cnt, 0) - bin_cnt
    # per-edge u16: local source | run-start marker | entry end
    E16 = (E + 15) // 16 * 16                         # phase 1 reads 16 edges per lane
    hbits = sl | (end.to(torch.int64) << 15)
    hbits[end_edge[run_first]] |= 1 << 14
    srcl = torch.zeros(E16, dtype=torch.int32, device=dev)
    srcl[:E] = hbits.to(torch.int32)
    srcl = srcl.to(torch.int16)                       # two's complement: bits 14, 15 kept
    del sl, hbits, end, rk, rstart
    # bin-major destination offsets
    pos = torch.arange(nent, device=dev) + run_delta[run_of_ent]
    n4 = (nent + 3) // 4 * 4 + PB_DUMMY                # + phase 1's per-wave dummy store slots
    dloc = torch.zeros(n4, dtype=torch.int32, device=dev)
    dloc[pos] = (ent_dst % bin_width).to(torch.int32)
    dloc = dloc.to(torch.int16)                       # < 32768: exact as int16
    del pos, ent_dst, ent_bin, ent_key
    # work units: a chunk is processed by ceil(E_chunk / wu_e) workgroups (wu_e ~ E / 4096:
    # ~8 rounds of the resident workgroups, so the hot chunks are no kernel tail on small
    # shards); tiles start on an entry boundary, never cross a work unit and are
    # min(tile, ~E_unit / 16) edges (>= 1024) so that the 8 waves of a unit all get work
    ce_lo = e_start[torch.searchsorted(ent_chunk, torch.arange(nch, device=dev))]
    ce_n = torch.diff(torch.cat([ce_lo, torch.tensor([E], dtype=torch.int64, device=dev)]))
    wu_e = max(1 << 15, E // 4096)
    tlen = torch.clamp((torch.clamp(ce_n, max=wu_e) + 15) // 16, min=min(1024, tile), max=tile)
    e_off = e_start - ce_lo[ent_chunk]
    M = wu_e // min(1024, tile) + 2                   # > tiles per work unit
    tk = ent_chunk * ((E // wu_e + 1) * M + 1) + (e_off // wu_e) * M + (e_off % wu_e) // tlen[ent_chunk]
    tnew = torch.ones(nent, dtype=torch.bool, device=dev)
    tnew[1:] = tk[1:] != tk[:-1]
    tile_ent = torch.nonzero(tnew).flatten()
    tile_e = torch.cat([e_start[tile_ent], torch.tensor([E], dtype=torch.int64, device=dev)])
    tile_chunk = ent_chunk[tile_ent]
    chunk_tile = torch.searchsorted(tile_chunk, torch.arange(nch + 1, device=dev))
    wk = tile_chunk * (E + 2) + e_off[tile_ent] // wu_e
    wnew = torch.ones_like(wk, dtype=torch.bool)
    wnew[1:] = wk[1:] != wk[:-1]
    wu_first = torch.nonzero(wnew).flatten()
    wu_tile = torch.cat([wu_first, torch.tensor([tile_ent.numel()], dtype=torch.int64, device=dev)])
    wu_chunk = tile_chunk[wu_first]
    del wk, wnew, wu_first
    tile_run = torch.searchsorted(run_first, tile_ent) - chunk_run[tile_chunk]
    del tk, tnew, e_start, ce_lo, ce_n, tlen, e_off, ent_chunk
    # the bounds the kernels rely on (checked once, here)
    assert int(tile_e[-1]) <= srcl.numel() and int((slo + ns).max()) <= n_src
    assert run_first.numel() == int(chunk_run[-1])
    # work items: each bin's contiguous entry range, hot bins cut into ~cap pieces
    (wb, wl, slab_h, sp_bin, sp_first, sp_cnt), nslab = _work_items(bin_cnt, bin_lo, nent, items, min_piece)
    return BlockedLayout(srcl, i64(tile_e), i32(tile_ent), i32(tile_run), i32(chunk_tile),
                         i32(wu_tile), i32(wu_chunk), i32(slo),
                         i32(ns), i32(chunk_run), i32(run_delta),
                         torch.zeros(n4, dtype=torch.float32, device=dev), dloc,
                         i32(wb), i64(wl), i32(slab_h),
                         torch.zeros(max(nslab, 1) * bin_width, dtype=torch.int64, device=dev),
                         i32(sp_bin), i32(sp_first), i32(sp_cnt), bin_width, nl, nch, nent, n_src,
                         max_indeg, int((chunk_run[1:] - chunk_run[:-1]).max().item()),
                         torch.zeros(1, dtype=torch.float64, device=dev),
                         int((slo[wu_chunk] < src_split).sum().item()) if src_split is not None else 0,
                         tuple(int((slo[wu_chunk] < b).sum().item()) for b in splits))


# ------------------------------------------------------------------ native build
@dataclass
class NativeGraph:
    """A rank's PageRank adjacency built natively from raw edge chunks (build_native):
    the K4b layout over the [own slice | ghosts] source index space, the deduplicated
    out-degree of every local source, and the ghost list (W > 1). Stands in for the
    (dst, src)-sorted :class:`GraphShard` of the blocked path; :meth:`to_shard` rebuilds
    that form (pull SpMV, witnesses) from the kept keys."""
    layout: BlockedLayout
    n_edges: int
    v_lo: int
    v_hi: int
    n_vertices: int
    slice_size: int
    outdeg_loc: torch.Tensor            # int32 [sl + n_ghost]: distinct out-edges per local source
    ghosts: torch.Tensor | None         # int64 sorted global ids of the remote sources (W > 1)
    recv_counts: list                   # ghosts per owner rank
    keys: torch.Tensor | None = None    # sorted keys with duplicates (kept for to_shard)
    n_keys: int = 0
    key_shift: int = 0
    dbits: int = 0
    blk_base: torch.Tensor | None = None
    new_id: torch.Tensor | None = None

    @property
    def n_local(self) -> int:
        return self.v_hi - self.v_lo

    @property
    def n_ghost(self) -> int:
        return 0 if self.ghosts is None else int(self.ghosts.numel())

    def to_shard(self) -> GraphShard:
        """The (dst, src)-sorted shard with GLOBAL source ids (needs the kept keys)."""
        if self.keys is None:
            raise ValueError("NativeGraph.to_shard needs the keys (build_native(keep_keys=True))")
        K = torch.unique_consecutive(self.keys[: self.n_keys])
        blk = K >> self.key_shift
        dl = (K >> SRC_BITS) & ((1 << self.dbits) - 1)
        li = self.blk_base[blk] + (K & (SRC_SPAN - 1))
        sl = self.slice_size
        if self.ghosts is not None:
            gs = torch.where(li < sl, li + self.v_lo,
                             self.ghosts[(li - sl).clamp(0, max(self.n_ghost - 1, 0))])
        else:
            gs = li + self.v_lo
        key = torch.sort((dl << 32) | gs).values
        sh = _shard_from_keys(key, self.v_lo, self.v_hi, self.n_vertices, sl)
        sh.new_id = self.new_id
        return sh


SRC_BITS = 13            # log2(SRC_SPAN)


def _popcount32(x: torch.Tensor) -> torch.Tensor:
    x = x.to(torch.int64) & 0xFFFFFFFF
    x = x - ((x >> 1) & 0x55555555)
    x = (x & 0x33333333) + ((x >> 2) & 0x33333333)
    x = (x + (x >> 4)) & 0x0F0F0F0F
    return ((x * 0x01010101) & 0xFFFFFFFF) >> 24


# phase marks of the native build (HIP events; None = off): build_phase_spans() turns the
# recorded marks into {phase: ms} after a device sync (bench diagnostics)
build_marks: list | None = None


def _mark(name: str):
    """A phase boundary: a HIP event, or (DALGO_BUILD_SYNC=1, diagnostics) a device sync
    and the host clock, so host-side costs land in the phase that causes them."""
    if build_marks is not None and torch.cuda.is_available():
        import os
        if os.environ.get("DALGO_BUILD_SYNC") == "1":
            import time
            torch.cuda.synchronize()
            build_marks.append((name, time.perf_counter()))
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        build_marks.append((name, e))


def build_phase_spans() -> dict:
    out = {}
    if build_marks:
        for (_, a), (name, b) in zip(build_marks[:-1], build_marks[1:]):
            dt = (b - a) * 1e3 if isinstance(a, float) else a.elapsed_time(b)
            out[name] = out.get(name, 0.0) + dt
    return out


def sort_split_bits(nbits: int) -> int:
    """Low key bits left to the in-place run sort (graph_build.hip gb_run_sort): the radix
    sort covers the bits above the source offset in whole 8-bit passes, extended down into
    the offset as far as its last pass has room (12 of 52 bits at scale 26)."""
    if nbits <= SRC_BITS:
        return 0
    passes = (nbits - SRC_BITS + 7) // 8
    return max(0, nbits - 8 * passes)


def build_native(edges: list, n_vertices: int, rank: int, world: int, new_id: torch.Tensor | None = None,
                 bin_width: int = 16384, tile: int = 16384, items: int | None = None,
                 min_piece: int = 1 << 14, keep_keys: bool = False,
                 packed: torch.Tensor | None = None, packed_src_new: bool = False) -> NativeGraph:
    """``distinct().groupByKey()`` of graph_computation/pagerank.py:41 straight into the
    K4b layout, on the device (csrc/kernels/graph_build.hip): relabel + keep this rank's
    destinations + pack one (block, destination, source offset) key per edge, ONE radix
    sort over the key's bits, unique, then single passes for the per-edge source offsets,
    the entries and their runs / tiles. Same layout as :func:`build_blocked` over the
    (dst, src)-sorted shard (chunks = whole 8192-source blocks, no edge cut).

    edges: list of (src, dst) int32 GPU chunks of GLOBAL ids (before ``new_id``).
    packed (one rank): the same edges as (src << 32 | dst) int64 words in any order
    (:func:`partition_edges`: partitioned on the source), read instead of ``edges``;
    packed_src_new: their sources are already relabelled (:func:`relabel_partition_dst`)."""
    if bin_width not in (8192, 16384):
        raise ValueError("bin_width must be 8192 or 16384")
    if items is None:
        items = pb_items(world)
    ops = _ext.ops()
    dev = edges[0][0].device
    N, W = n_vertices, world
    sl = vertex_slices(N, W)
    v_lo, v_hi = rank * sl, min(N, (rank + 1) * sl)
    nl = v_hi - v_lo
    dbits = max(1, (max(nl, 1) - 1).bit_length())
    S = SRC_SPAN
    i64 = dict(dtype=torch.int64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    nid = new_id.to(torch.int32).contiguous() if new_id is not None else None
    # ---- phase 0: kept edges per key block (+ remote-source marks, W > 1)
    nwords = (N + 31) // 32 + 1
    bitmap = torch.empty(nwords, **i32) if W > 1 else None
    nbs = [(int(s.numel()) + 16383) // 16384 for s, _ in edges]     # graph_build.hip kKeyR
    if W > 1:
        counts = torch.empty(sum(nbs), **i32)
        # remote sources: one byte per id (plain stores), packed into the bitmap after
        marks = torch.zeros(max(32 * nwords, sl * W), dtype=torch.uint8, device=dev)
        o = 0
        for (s, d), nb in zip(edges, nbs):
            ops.gb_keys(s, d, nid, v_lo, v_hi, sl, W, rank, dbits, 0, marks, counts[o:o + nb], None, 0,
                        None, None, None, None)
            o += nb
        ops.gb_bytes_to_bits(marks, bitmap)
        del marks
        c64 = counts.to(torch.int64)
        offsets = torch.cumsum(c64, 0) - c64
        total = int(c64.sum().item())
        pc = _popcount32(bitmap)
        word_prefix = torch.cumsum(pc, 0) - pc
        n_ghost = int(pc.sum().item())
        ghosts = torch.empty(n_ghost, **i64)
        ops.gb_bitmap_ids(bitmap, word_prefix, ghosts)     # sorted ids of the set bits
        # ghosts per owner: the sorted list cut at the slice boundaries
        cuts = torch.searchsorted(ghosts, torch.arange(W + 1, **i64) * sl)
        recv_counts = [int(x) for x in torch.diff(cuts).tolist()]
    else:
        total = sum(int(s.numel()) for s, _ in edges)
        offsets, word_prefix, ghosts, n_ghost, recv_counts = None, None, None, 0, [0]
    _mark("count")
    # ---- segments of the local source index space: own [0, nl), then each peer's ghosts
    seg_start = [0] * W
    seg_end = [0] * W
    seg_blk0 = [0] * W
    seg_end[rank] = nl
    nblk = (nl + S - 1) // S
    goff = 0
    for p in range(W):
        if p == rank:
            continue
        seg_start[p] = sl + goff
        goff += recv_counts[p]
        seg_end[p] = sl + goff
        seg_blk0[p] = nblk
        nblk += (recv_counts[p] + S - 1) // S
    blk_base = torch.empty(max(nblk, 1), **i64)
    blk_end = torch.empty(max(nblk, 1), **i64)
    for p in range(W):
        nb = ((seg_end[p] - seg_start[p]) + S - 1) // S
        if nb:
            b0 = seg_blk0[p]
            base = seg_start[p] + S * torch.arange(nb, **i64)
            blk_base[b0:b0 + nb] = base
            blk_end[b0:b0 + nb] = seg_end[p]
    blk_bits = max(1, (max(nblk, 1) - 1).bit_length())
    shift = dbits + SRC_BITS
    nbits = shift + blk_bits
    assert nbits <= 63, "key does not fit 63 bits"
    st = torch.tensor(seg_start, **i64)
    sb = torch.tensor(seg_blk0, **i64)
    _mark("segments")
    # ---- phase 1: keys
    keys = torch.empty(max(total, 1), **i64)
    from_packed = packed is not None
    if from_packed:
        if W != 1 or packed.numel() != total:
            raise ValueError("build_native: packed edges are the one-rank path over every edge")
        ops.gb_keys_packed(packed, nid, N, dbits, keys, int(bool(packed_src_new)))
        del packed
    o, base_all = 0, 0
    for (s, d), nb in zip(edges, nbs):
        if from_packed:
            break
        ops.gb_keys(s, d, nid, v_lo, v_hi, sl, W, rank, dbits, 1, bitmap, None,
                    offsets[o:o + nb] if offsets is not None else None, base_all, keys,
                    word_prefix, st, sb)
        o += nb
        base_all += int(s.numel())
    del bitmap, word_prefix, offsets
    _mark("keys")
    K = torch.empty_like(keys)
    if total:
        # whole radix passes over the bits above the source offset (5 instead of 7 at scale
        # 26: bits 12..51), then each run of keys equal there sorted in place on the rest
        lo = sort_split_bits(nbits)
        ops.gb_sort(keys, total, nbits, K, lo)
        if lo:
            ops.gb_run_sort(K, total, lo)
    del keys
    _mark("sort")
    n_src_loc = (sl + n_ghost) if W > 1 else max(N, 1)
    outdeg_loc = torch.zeros(n_src_loc, **i32)
    if total == 0:
        shard = GraphShard(torch.full((4,), -1, **i32), torch.full((4,), -1, **i32), 0, v_lo, v_hi, N, sl)
        lay = build_blocked(shard, bin_width, 1 << 40, tile, items, min_piece)
        return NativeGraph(lay, 0, v_lo, v_hi, N, sl, outdeg_loc, ghosts, recv_counts,
                           K if keep_keys else None, 0, shift, dbits, blk_base, new_id)
    # ---- decode (dedup folded in): per distinct edge the source offset + entry-end bit,
    # the entries, the distinct out-degrees
    nbd = int(ops.gb_decode_blocks(total))            # graph_build.hip kDecR keys per block
    counts = torch.empty(2 * nbd, **i64)
    ops.gb_decode(K, total, shift, dbits, blk_base, 0, counts, outdeg_loc, None, None, None, None, None)
    # (scanned as two rows: torch's scan down the 2-column [nbd, 2] view ran 2.6 ms at scale
    # 26 -- one thread per column -- profiles/round6/r6_48)
    ct = counts.view(nbd, 2).t().contiguous()
    offsets = (torch.cumsum(ct, 1) - ct).t()
    E, nent = (int(x) for x in ct.sum(1).tolist())
    E16 = (E + 15) // 16 * 16
    srcl = torch.empty(E16, dtype=torch.int16, device=dev)   # the decode writes [0, E)
    srcl[E:].zero_()
    ent_end = torch.empty(nent, **i64)
    ent_blk = torch.empty(nent, **i32)
    ent_dst = torch.empty(nent, **i32)
    ops.gb_decode(K, total, shift, dbits, blk_base, 1, None, None, offsets.contiguous().view(-1), srcl,
                  ent_end, ent_blk, ent_dst)
    del counts, offsets
    if not keep_keys:
        del K
        K = None
    _mark("decode")
    # ---- entries: run / chunk starts, run-start bits, bin-major places, tile starts
    bshift = bin_width.bit_length() - 1
    nbins = max(1, (nl + bin_width - 1) // bin_width)
    nblk_k = max(nblk, 1)
    wu_e = max(1 << 15, E // PB_UNITS)
    n4 = (nent + 3) // 4 * 4 + PB_DUMMY
    # every entry's bin-major place is written once below (a bijection onto [0, nent)):
    # only the padding is cleared
    dloc = torch.empty(n4, dtype=torch.int16, device=dev)
    dloc[nent:].zero_()
    assert nent < (1 << 31) - 8
    if nblk_k * nbins <= CELL_CAP:
        # runs = the non-empty cells of the (block, bin) matrix (graph_build.hip gb_cell_*)
        ncell = nblk_k * nbins
        C = torch.zeros(ncell, **i32)
        ops.gb_cell_count(ent_blk, ent_dst, bshift, nblk_k, nbins, C)
        T = torch.empty(nblk_k, **i64)
        R = torch.empty(nblk_k, **i64)
        ops.gb_cell_rows(C, nblk_k, nbins, T, R)
        RE = torch.cumsum(T, 0) - T                       # first entry of every block
        RR = torch.cumsum(R, 0) - R                       # first run of every block
        nz = T > 0
        CI = (torch.cumsum(nz, 0) - nz.long()).to(torch.int32)   # chunk of a non-empty block
        nch, nruns, max_runs = (int(x) for x in torch.stack([nz.sum(), R.sum(), R.max()]).tolist())
        CM = torch.empty(ncell, **i32)
        RID = torch.empty(ncell, **i32)
        ops.gb_cell_scan(C, nblk_k, nbins, RE, RR, CM, RID)
        G = 64
        ng = (nblk_k + G - 1) // G
        P = torch.empty((ng, nbins), **i64)
        ops.gb_cell_colsum(C, nblk_k, nbins, G, P)
        bin_cnt = P.sum(0)
        bin_lo = torch.cumsum(bin_cnt, 0) - bin_cnt
        Poff = torch.cumsum(P, 0) - P + bin_lo
        run_delta = torch.empty(nruns, **i32)
        run_chunk = torch.empty(nruns, **i32)
        run_first = torch.empty(nruns, **i64)
        ops.gb_cell_place(C, CM, RID, nblk_k, nbins, G, Poff, CI, run_delta, run_chunk, run_first)
        del C, P, Poff
        chunk_blk = torch.nonzero(nz).flatten()
        chunk_first = RE[chunk_blk]
        chunk_run = torch.cat([RR[chunk_blk], torch.tensor([nruns], **i64)])
        _mark("entries_runs")
        ce_lo = torch.where(chunk_first > 0, ent_end[(chunk_first - 1).clamp_min(0)] + 1,
                            torch.zeros_like(chunk_first))
        ce_n = torch.diff(torch.cat([ce_lo, torch.tensor([E], **i64)]))
        tlen = torch.clamp((torch.clamp(ce_n, max=wu_e) + PB_TILES - 1) // PB_TILES, min=min(1024, tile), max=tile)
        # tile starts: at most one per chunk start, per work-unit boundary and per tlen
        # boundary inside a unit
        cap_t = int((1 + (ce_n + wu_e - 1) // wu_e + (ce_n + tlen - 1) // tlen).sum().item())
        tiles_l = torch.empty(max(cap_t, 1), **i32)
        n_t = torch.zeros(1, **i64)
        ops.gb_entry_cells(ent_blk, ent_dst, ent_end, bshift, nblk_k, nbins, CM, RID, run_delta, RE, CI,
                           ce_lo, tlen, wu_e, bin_width - 1, dloc, tiles_l, n_t, srcl)
        del CM, RID, ent_dst, ent_blk, RE, RR, CI
        _mark("entry_place")
        nt = int(n_t.item())
        assert nt <= cap_t, (nt, cap_t)
        # (the build's own u64 radix sort: torch.sort at this size took 32 ms on its first
        # use in a process, profiles/round5/r5_31)
        tk = tiles_l[:nt].to(torch.int64)
        tile_ent = torch.empty_like(tk)
        if nt:
            ops.gb_sort(tk, nt, max(1, (nent - 1).bit_length()), tile_ent)
        del tiles_l, tk
    else:
        # matrix too large: per-entry flags, scans and a sort of the runs
        rs = torch.empty(nent, dtype=torch.uint8, device=dev)
        cs = torch.empty(nent, dtype=torch.uint8, device=dev)
        ops.gb_entry_flags(ent_blk, ent_dst, ent_end, bshift, rs, cs, srcl)
        run_first = torch.nonzero(rs).flatten()
        chunk_first = torch.nonzero(cs).flatten()
        nch = int(chunk_first.numel())
        nruns = int(run_first.numel())
        chunk_blk = ent_blk[chunk_first].to(torch.int64)
        run_of_ent = (torch.cumsum(rs, 0, dtype=torch.int32) - 1)
        del rs
        run_chunk = torch.searchsorted(chunk_first, run_first, right=True) - 1
        run_bin = (ent_dst[run_first] >> bshift).to(torch.int64)
        run_len = torch.diff(torch.cat([run_first, torch.tensor([nent], **i64)]))
        border = torch.argsort(run_bin * (nch + 1) + run_chunk)
        bm_start = torch.empty_like(run_first)
        bm_start[border] = torch.cumsum(run_len[border], 0) - run_len[border]
        run_delta = (bm_start - run_first).to(torch.int32)
        run_chunk = run_chunk.to(torch.int32)
        del bm_start, border
        chunk_run = torch.searchsorted(run_chunk.to(torch.int64), torch.arange(nch + 1, **i64))
        bin_cnt = torch.zeros(nbins, **i64).index_add_(0, run_bin, run_len)
        bin_lo = torch.cumsum(bin_cnt, 0) - bin_cnt
        max_runs = int((chunk_run[1:] - chunk_run[:-1]).max().item())
        _mark("entries_runs")
        # tiles / work units: a chunk is cut every wu_e edges into work units and every
        # tlen edges inside a unit into tiles, both on entry boundaries
        ce_lo = torch.where(chunk_first > 0, ent_end[(chunk_first - 1).clamp_min(0)] + 1,
                            torch.zeros_like(chunk_first))
        ce_n = torch.diff(torch.cat([ce_lo, torch.tensor([E], **i64)]))
        tlen = torch.clamp((torch.clamp(ce_n, max=wu_e) + PB_TILES - 1) // PB_TILES, min=min(1024, tile), max=tile)
        ts = torch.empty(nent, dtype=torch.uint8, device=dev)
        ops.gb_entry_place(ent_dst, ent_end, run_of_ent, run_delta, run_chunk, cs,
                           ce_lo, tlen, wu_e, bin_width - 1, dloc, ts)
        del run_of_ent, cs, ent_dst, ent_blk
        _mark("entry_place")
        tile_ent = torch.nonzero(ts).flatten()
        del ts
    assert nruns < (1 << 31)
    _mark("tile_select")
    e_start_t = torch.where(tile_ent > 0, ent_end[(tile_ent - 1).clamp_min(0)] + 1, torch.zeros_like(tile_ent))
    del ent_end
    tile_e = torch.cat([e_start_t, torch.tensor([E], **i64)])
    tile_chunk = torch.searchsorted(chunk_first, tile_ent, right=True) - 1
    chunk_tile = torch.searchsorted(tile_chunk, torch.arange(nch + 1, **i64))
    wk = tile_chunk * (E + 2) + (e_start_t - ce_lo[tile_chunk]) // wu_e
    wnew = torch.ones_like(wk, dtype=torch.bool)
    wnew[1:] = wk[1:] != wk[:-1]
    wu_first = torch.nonzero(wnew).flatten()
    wu_tile = torch.cat([wu_first, torch.tensor([tile_ent.numel()], **i64)])
    wu_chunk = tile_chunk[wu_first]
    tile_run = torch.searchsorted(run_first, tile_ent) - chunk_run[tile_chunk]
    slo = blk_base[chunk_blk]
    ns = torch.clamp(blk_end[chunk_blk] - slo, max=S)
    n_src, ns_min, te_last = (int(x) for x in torch.stack([(slo + ns).max(), ns.min(), tile_e[-1]]).tolist())
    assert te_last <= srcl.numel() and ns_min >= 1
    _mark("tiles")
    # ---- phase-2 work items (as build_blocked)
    (wb, wl, slab_h, sp_bin, sp_first, sp_cnt), nslab = _work_items(bin_cnt, bin_lo, nent, items, min_piece)
    _mark("work_split")
    it = lambda x: torch.tensor(x, **i32)
    c32 = lambda x: x.to(torch.int32).contiguous()
    splits = sorted({int(x) for x in seg_start if x > 0})
    # entry values: phase 1 writes every entry [0, nent) before phase 2 reads it, so only
    # the padding is cleared (a full 1.9 GB fill was 0.26 ms of the scale-26 build)
    val = torch.empty(n4, dtype=torch.float32, device=dev)
    val[nent:].zero_()
    lay = BlockedLayout(srcl, tile_e.contiguous(), c32(tile_ent), c32(tile_run), c32(chunk_tile),
                        c32(wu_tile), c32(wu_chunk), c32(slo), c32(ns), c32(chunk_run), c32(run_delta),
                        val, dloc,
                        c32(wb), wl.to(device=dev).contiguous(), c32(slab_h),
                        torch.zeros(max(nslab, 1) * bin_width, **i64),
                        c32(sp_bin), c32(sp_first), c32(sp_cnt), bin_width, nl, nch, nent, n_src,
                        0, max_runs, torch.zeros(1, dtype=torch.float64, device=dev),
                        int((slo[wu_chunk] < sl).sum().item()) if W > 1 else 0,
                        tuple(int((slo[wu_chunk] < b).sum().item()) for b in splits))
    _mark("work_items")
    return NativeGraph(lay, E, v_lo, v_hi, N, sl, outdeg_loc, ghosts, recv_counts, K, total, shift, dbits,
                       blk_base, new_id)


def pb_spmv(lay: BlockedLayout, c_full: torch.Tensor, acc: torch.Tensor, pres: torch.Tensor,
            update: dict | None = None, wu_range: tuple | None = None, phases: int = 3):
    """Same result as :func:`pr_spmv` (every acc / pres entry is written: no pre-zeroing).
    The GPU sums are exact u64 fixed-point sums (order independent) rounded to f32 once;
    their scale 2^K comes from this call's data (phase 1 sums the present c values it
    stages: no destination sum can exceed that), computed on the device (no host sync).
    ``update``: dict(outdeg, q, invN, mode, r, c, dangling_in, dangling_out) fuses
    :func:`pr_update` into the epilogue (acc / pres are then not written).
    ``phases``: 1 = phase 1 over the work units ``wu_range`` only (the calls of one
    product must cover all units, the first starting at 0), 2 = phase 2 only, 3 = both."""
    if c_full.numel() < lay.n_src or acc.numel() != lay.n_local:
        raise ValueError("pb_spmv: c_full / acc do not match the layout")
    if c_full.is_cuda:
        u = update or {}
        _ext.ops().pb_spmv(lay.srcl, lay.tile_e, lay.tile_ent, lay.tile_run, lay.wu_tile, lay.wu_chunk,
                           lay.chunk_slo, lay.chunk_ns, lay.chunk_run, lay.run_delta, c_full,
                           lay.val, lay.dloc, lay.wi_bin, lay.wi_lo, lay.wi_slab, lay.bin_width,
                           lay.max_runs, lay.bound, acc, pres, lay.slab, lay.split_bin,
                           lay.split_first, lay.split_count, u.get("outdeg"), float(u.get("q", 0.0)),
                           float(u.get("invN", 0.0)), int(u.get("mode", 0)), u.get("dangling_in"),
                           u.get("r"), u.get("c"), u.get("dangling_out"),
                           int(wu_range[0]) if wu_range else 0,
                           int(wu_range[1]) if wu_range else 2147483647, int(phases))
        return
    if not (phases & 2):          # CPU reference: everything happens in the phase-2 call
        return
    acc.zero_()
    pres.zero_()
    # CPU reference of the two phases, decoding the same per-edge bits as the kernels
    if lay.n_chunks > 0:
        _pb_cpu(lay, c_full, acc, pres)
    if update is not None:
        pr_update(acc, pres, update["outdeg"], update["q"], update["invN"], update["mode"],
                  update["r"], update["c"], update.get("dangling_in"), update.get("dangling_out"))


def _pb_cpu(lay: BlockedLayout, c_full: torch.Tensor, acc: torch.Tensor, pres: torch.Tensor):
    E = int(lay.tile_e[-1])
    h = (lay.srcl[:E].to(torch.int32) & 0xFFFF).long()
    nt = lay.tile_e.numel() - 1
    tile_of_e = torch.repeat_interleave(torch.arange(nt), (lay.tile_e[1:] - lay.tile_e[:-1]))
    chunk_of_tile = torch.repeat_interleave(torch.arange(lay.n_chunks),
                                            (lay.chunk_tile[1:] - lay.chunk_tile[:-1]).long())
    ch = chunk_of_tile[tile_of_e]
    cv = c_full[lay.chunk_slo.long()[ch] + (h & (SRC_SPAN - 1))]
    end = (h >> 15) & 1
    ent = torch.cumsum(end, 0) - end                  # chunk-major entry of each edge
    v = torch.zeros(lay.n_entries, dtype=c_full.dtype)
    v.index_add_(0, ent, cv.clamp_min(0))
    hit = torch.zeros(lay.n_entries, dtype=torch.int64)
    hit.index_add_(0, ent, (cv >= 0).long())
    # run of each entry: run-start markers on the entries' end edges, counted per chunk
    ee = torch.nonzero(end).flatten()
    mark = (h[ee] >> 14) & 1
    ent_ch = ch[ee]
    ordinal = torch.cumsum(mark, 0) - 1               # global run index (chunk-major)
    assert bool((ordinal >= lay.chunk_run.long()[ent_ch]).all())
    pos = torch.arange(lay.n_entries) + lay.run_delta.long()[ordinal]
    vb = torch.zeros(lay.n_entries, dtype=c_full.dtype)
    hb = torch.zeros(lay.n_entries, dtype=torch.int64)
    vb[pos] = v
    hb[pos] = hit
    dl = (lay.dloc[:lay.n_entries].to(torch.int32) & 0xFFFF).long()
    b_of = torch.repeat_interleave(lay.wi_bin.long(), lay.wi_lo[1:] - lay.wi_lo[:-1])
    dd = b_of * lay.bin_width + dl
    acc.index_add_(0, dd, vb.to(acc.dtype))
    ph = torch.zeros_like(pres)
    ph.index_add_(0, dd, (hb > 0).to(pres.dtype))
    pres.copy_((ph > 0).to(pres.dtype))


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
