"""graph_computation/pagerank.py entry logic."""
from __future__ import annotations

import torch

from dalgo.models.pagerank import PageRank, PageRankConfig
from dalgo.models.transitive_closure import compact_ids
from dalgo.ops import graph as G
from dalgo.parallel import runtime
from dalgo.utils import checkpoint, obs
from dalgo.utils.cli import add_ckpt_args, common_parser, init_from_args

TOY_EDGES = [(1, 2), (1, 3), (2, 3), (3, 1)]   # pagerank.py:35-38


def load_edges(path: str):
    import numpy as np
    arr = np.loadtxt(path, dtype=np.int64, delimiter=None, ndmin=2)
    return torch.from_numpy(arr[:, 0]).to(torch.int32), torch.from_numpy(arr[:, 1]).to(torch.int32)


def degree_order(scale: int, edge_factor: int, rank: int, world: int, device, seed: int = 1,
                 chunk: int = 1 << 26) -> torch.Tensor:
    """new_id[old]: vertices ranked by descending out-degree (ties by id), DEALT round-robin
    over the W destination slices.

    Gather locality for the pull SpMV: the contributions c[u] that the most edges read
    (high out-degree u) sit at the front of every slice, a cache-resident prefix of each.
    Dealing instead of cutting the ranked list into W contiguous pieces keeps the
    destination partition balanced: in R-MAT the in- and out-hubs coincide, and the
    contiguous cut gave slice 0 7x the mean in-edge count at W = 8 (88 % of the edges,
    scale 18; tests/test_cpu_algorithms.py::test_pagerank_degree_order_balanced).
    Every rank counts 1/W of the edge stream, one all-reduce.
    """
    from dalgo.parallel import comm
    n_vertices = 1 << scale
    n_edges = edge_factor * n_vertices
    deg = torch.zeros(n_vertices, dtype=torch.int64, device=device)
    chunks = list(range(0, n_edges, chunk))
    for i, off in enumerate(chunks):
        if i % world != rank:
            continue
        s, _ = G.rmat_edges(min(chunk, n_edges - off), scale, seed=seed, e_off=off, device=device)
        G.degree_count_(deg, s)
    comm.all_reduce_sum(deg)
    order = torch.argsort(-deg * n_vertices - torch.arange(n_vertices, device=device, dtype=torch.int64))
    return deal_ids(order, n_vertices, world).to(torch.int32)


def deal_ids(order: torch.Tensor, n_vertices: int, world: int) -> torch.Tensor:
    """new_id[old] for the ranked vertex list ``order`` (order[j] = j-th vertex): rank j
    goes to position j // W of slice j % W, snake order (odd rounds deal W-1 .. 0, so no
    slice always gets the heaviest vertex of a round), with the slices of
    G.vertex_slices (the last ones may be shorter); ranks past a full slice take the
    free positions in order. A bijection of [0, n_vertices)."""
    dev = order.device
    if world == 1:                       # rank j -> position j
        new_id = torch.empty(n_vertices, dtype=torch.int64, device=dev)
        new_id[order] = torch.arange(n_vertices, device=dev, dtype=torch.int64)
        return new_id
    sl = G.vertex_slices(n_vertices, world)
    if dev.type == "cuda" and sl * world == n_vertices:
        # every slice full: one scatter kernel (graph_build.hip gb_deal)
        from dalgo.ops import _ext
        new_id = torch.empty(n_vertices, dtype=torch.int32, device=dev)
        _ext.ops().gb_deal(order.to(torch.int64).contiguous(), world, sl, 0, new_id)
        return new_id
    j = torch.arange(n_vertices, device=dev, dtype=torch.int64)
    p = j // world
    r = torch.where(p % 2 == 0, j % world, world - 1 - j % world)
    size = torch.clamp(n_vertices - torch.arange(world, device=dev, dtype=torch.int64) * sl, 0, sl)
    pos = r * sl + p
    ok = p < size[r]
    if not bool(ok.all()):
        used = torch.zeros(n_vertices, dtype=torch.bool, device=dev)
        used[pos[ok]] = True
        pos = pos.clone()
        pos[~ok] = torch.nonzero(~used).flatten()[: int((~ok).sum())]
    new_id = torch.empty(n_vertices, dtype=torch.int64, device=dev)
    new_id[order] = pos
    return new_id


def rmat_input(scale: int, edge_factor: int, device, seed: int = 1, chunk: int = 1 << 26):
    """The whole R-MAT edge stream as a list of (src, dst) int32 chunks (the job's input:
    the reference's ``parallelize(links)``, graph_computation/pagerank.py:35-38)."""
    n_edges = edge_factor * (1 << scale)
    from dalgo.parallel import runtime
    parts = []
    for off in range(0, n_edges, chunk):
        runtime.heartbeat()   # long generation is progress (stall watchdog)
        parts.append(G.rmat_edges(min(chunk, n_edges - off), scale, seed=seed, e_off=off,
                                  device=device))
    return parts, n_edges


def degree_order_from(edges: list, scale: int, rank: int, world: int, device) -> torch.Tensor:
    """:func:`degree_order` over a given chunk list (every rank counts chunks i % W == rank,
    one all-reduce)."""
    from dalgo.parallel import comm
    n_vertices = 1 << scale
    deg = torch.zeros(n_vertices, dtype=torch.int32, device=device)
    mine = [s for i, (s, _) in enumerate(edges) if i % world == rank]
    if mine and deg.is_cuda:
        # one radix sort of this rank's sources + run lengths (graph_build.hip)
        ids = torch.cat(mine) if len(mine) > 1 else mine[0]
        G.degree_sorted_(deg, ids, scale)
        del ids
    else:
        for s in mine:
            G.degree_count_(deg, s)
    comm.all_reduce_sum(deg)
    G._mark("degree_count")
    return degree_new_id(deg, n_vertices, world)


def degree_new_id(deg: torch.Tensor, n_vertices: int, world: int) -> torch.Tensor:
    """int32 new_id of the degree relabeling, ``deal_ids(rank_by_degree(deg), n, W)``. GPU with
    full slices (every W dividing 2^scale, W = 1 included): the ranking keys in one kernel,
    the sort over the degree bits, then the snake deal straight from the sorted keys (their
    id bits masked in the scatter) -- 3 kernels and a sort instead of ~10 (graph_build.hip
    gb_rank_keys, gb_deal)."""
    sl = G.vertex_slices(n_vertices, world)
    if not (deg.is_cuda and sl * world == n_vertices and deg.numel() == n_vertices and n_vertices > 1):
        return deal_ids(rank_by_degree(deg), n_vertices, world).to(torch.int32)
    from dalgo.ops import _ext
    ops = _ext.ops()
    deg = deg.to(torch.int32).contiguous()
    dmax = int(deg.max().item())
    dbits = max(1, dmax.bit_length())
    ibits = max(1, (n_vertices - 1).bit_length())
    keys = torch.empty(n_vertices, dtype=torch.int64, device=deg.device)
    ops.gb_rank_keys(deg, dmax, ibits, keys)
    out = torch.empty_like(keys)
    # (capping the degree bits at 16 -- 2 radix passes instead of 3 at scale 26 -- and
    # re-ranking the few vertices above the cap with torch was no faster: r6_31)
    ops.gb_sort(keys, n_vertices, dbits + ibits, out, ibits)
    del keys
    new_id = torch.empty(n_vertices, dtype=torch.int32, device=deg.device)
    ops.gb_deal(out, world, sl, ibits, new_id)
    return new_id


def rank_by_degree(deg: torch.Tensor) -> torch.Tensor:
    """Vertex ids by descending degree, ties by descending id (argsort of -deg * n - id).
    GPU: one rocPRIM radix sort of ((max - deg) << b | id) keys laid out in descending id
    order, over the degree bits only (stable: equal degrees keep that order; 3 passes at
    R-MAT scale 26 instead of 6 over all bits; graph_build.hip gb_sort)."""
    n = deg.numel()
    if deg.is_cuda:
        from dalgo.ops import _ext
        dmax = int(deg.max().item()) if n else 0
        dbits = max(1, dmax.bit_length())
        ibits = max(1, (n - 1).bit_length())
        rid = torch.arange(n - 1, -1, -1, device=deg.device, dtype=torch.int64)   # descending ids
        keys = ((dmax - deg.to(torch.int64).flip(0)) << ibits) | rid
        out = torch.empty_like(keys)
        _ext.ops().gb_sort(keys, n, dbits + ibits, out, ibits)
        return out & ((1 << ibits) - 1)
    ids = torch.arange(n, device=deg.device, dtype=torch.int64)
    return torch.argsort(-deg.to(torch.int64) * n - ids)


def build_rmat_shard(edges: list, scale: int, rank: int, world: int, device, reorder: bool = True,
                     seed: int = 1):
    """This rank's shard of the given R-MAT edge chunks: optional degree relabeling, keep
    the destinations of this rank's slice, sort + dedup (``distinct().groupByKey()``)."""
    n_vertices = 1 << scale
    sl = G.vertex_slices(n_vertices, world)
    v_lo, v_hi = rank * sl, min(n_vertices, (rank + 1) * sl)
    new_id = degree_order_from(edges, scale, rank, world, device) if reorder else None
    parts = []
    for s, d in edges:
        if new_id is not None:
            s = new_id[s.long()]
            d = new_id[d.long()]
        keep = (d >= v_lo) & (d < v_hi)
        parts.append((s[keep], d[keep] - v_lo))
        del s, d
    shard = G.merge_shards(parts, v_lo, v_hi, n_vertices, sl)
    shard.new_id = new_id
    return shard


def build_rmat_native(edges: list, scale: int, rank: int, world: int, device, reorder: bool = True,
                      keep_keys: bool = False, bin_width: int = 16384, tile: int = 16384):
    """This rank's K4b-ready adjacency of the given R-MAT edge chunks, built natively
    (dalgo.ops.graph.build_native): degree relabeling, destination filter, dedup and the
    blocked layout without the (dst, src)-sorted intermediate shard. One rank with
    relabeling: the (src, dst) pairs are packed and partitioned on the high source bits
    first (the degree count's own partition), the sources relabelled there (32 KB slices of
    the table per bucket), then partitioned on the high destination bits, so the key pass
    relabels the destinations from such slices too: no random table gathers."""
    G._mark("start")
    packed = None
    if reorder and world == 1 and torch.device(device).type == "cuda" and scale > G.BUCKET_BITS:
        packed, deg = G.partition_edges(edges, scale)
        G._mark("degree_count")
        new_id = degree_new_id(deg, 1 << scale, 1)
        del deg
        G._mark("deal_ids")
        packed = G.relabel_partition_dst(packed, new_id, scale)
        G._mark("dst_partition")
    else:
        new_id = degree_order_from(edges, scale, rank, world, device) if reorder else None
        G._mark("deal_ids")
    return G.build_native(edges, 1 << scale, rank, world, new_id, bin_width=bin_width, tile=tile,
                          keep_keys=keep_keys, packed=packed, packed_src_new=packed is not None)


def edge_range(n_edges: int, rank: int, world: int) -> tuple[int, int]:
    """Rank's contiguous share [lo, hi) of an n_edges input stream."""
    return n_edges * rank // world, n_edges * (rank + 1) // world


def rmat_input_share(scale: int, edge_factor: int, rank: int, world: int, device, seed: int = 1):
    """This rank's E/W share of the R-MAT stream as ONE (src, dst) chunk: each rank holds
    (generates, or would load) only its part of the input, the reference's
    ``parallelize(links, n_slices)`` (graph_computation/pagerank.py:35-38)."""
    from dalgo.parallel import runtime
    n_edges = edge_factor * (1 << scale)
    lo, hi = edge_range(n_edges, rank, world)
    runtime.heartbeat()
    return [G.rmat_edges(hi - lo, scale, seed=seed, e_off=lo, device=device)], n_edges


def degree_order_share(edges: list, scale: int, world: int, device) -> torch.Tensor:
    """:func:`degree_order` when every rank holds a disjoint share of the input: each rank
    counts the sources of ALL its chunks, one all-reduce of the degrees, the same ranking
    and dealing on every rank."""
    from dalgo.parallel import comm
    n_vertices = 1 << scale
    deg = torch.zeros(n_vertices, dtype=torch.int32, device=device)
    if edges and deg.is_cuda and scale > G.BUCKET_BITS + 2:
        ids = torch.cat([s for s, _ in edges]) if len(edges) > 1 else edges[0][0]
        G.degree_sorted_(deg, ids, scale)
        del ids
    else:
        for s, _ in edges:
            G.degree_count_(deg, s)
    comm.all_reduce_sum(deg)
    G._mark("degree_count")
    return degree_new_id(deg, n_vertices, world)


def shuffle_edges(edges: list, new_id: torch.Tensor | None, n_vertices: int, world: int):
    """``groupByKey`` over the ranks (graph_computation/pagerank.py:41): this rank's input
    edges relabelled through new_id and sent to the owners of their destinations in ONE
    uneven all_to_all of packed (src << 32 | dst) words (plus one of the counts). Returns
    the (src, dst) int32 edges whose destination this rank owns, global new ids."""
    packs, counts = [], []
    for s, d in edges:
        p, c = G.owner_partition(s, d, new_id, n_vertices, world)
        packs.append(p)
        counts.append(c)
    if len(packs) == 1:
        packed, send = packs[0], counts[0]
    else:   # several chunks: owner-major concatenation
        pieces = []
        for o in range(world):
            for p, c in zip(packs, counts):
                a = sum(c[:o])
                pieces.append(p[a:a + c[o]])
        packed = torch.cat(pieces)
        send = [sum(c[o] for c in counts) for o in range(world)]
    del packs
    G._mark("owner_partition")
    return exchange_owner_major(packed, send)


def exchange_owner_major(packed: torch.Tensor, send: list):
    """The shuffle's collective: owner-major packed words (``send[o]`` for rank o) through ONE
    uneven all_to_all (plus one of the counts). Returns the received (src, dst) int32 edges."""
    from dalgo.parallel import comm
    dev = packed.device
    st = torch.tensor(send, dtype=torch.int64, device=dev)
    rt_ = torch.empty_like(st)
    comm.all_to_all_single(rt_, st)
    recv = [int(x) for x in rt_.tolist()]
    out = torch.empty(max(sum(recv), 1), dtype=torch.int64, device=dev)
    comm.all_to_all_single(out[: sum(recv)], packed, recv, send)
    del packed
    G._mark("all_to_all")
    return G.unpack_edges(out[: sum(recv)])


def build_rmat_sharded(edges: list, scale: int, rank: int, world: int, device, reorder: bool = True,
                       native: bool | None = None, keep_keys: bool = False, bin_width: int = 16384,
                       tile: int = 16384):
    """This rank's PageRank adjacency when every rank holds only E/W input edges: degree
    relabeling from one all-reduce of the share degrees, the shuffle of the relabelled
    edges to their destination owners (:func:`shuffle_edges`), then the build over what
    arrived -- native K4b layout on GPUs (dalgo.ops.graph.build_native, no relabeling left
    to do), the torch (dst, src) shard otherwise. Per rank O(E / W) work but the O(N)
    ranking of the degree order."""
    G._mark("start")
    n_vertices = 1 << scale
    if reorder and torch.device(device).type == "cuda" and scale > G.BUCKET_BITS and edges:
        # the one-rank build's partitions over this rank's share: sources partitioned on
        # their high bits (the degree count's own pass), relabelled bucket by bucket, then
        # grouped on the destination bits so the owner pass relabels destinations from
        # L2-resident slices of new_id (the direct path's random gathers over the whole table
        # were 5.2 of its 5.9 ms at the W = 8 share, profiles/round6/r6_23)
        from dalgo.parallel import comm
        packed, deg = G.partition_edges(edges, scale)
        comm.all_reduce_sum(deg)
        G._mark("degree_count")
        new_id = degree_new_id(deg, n_vertices, world)
        del deg
        G._mark("deal_ids")
        packed = G.relabel_partition_dst(packed, new_id, scale)
        G._mark("dst_partition")
        packed, send = G.owner_partition_packed(packed, new_id, n_vertices, world)
        G._mark("owner_partition")
        s, d = exchange_owner_major(packed, send)
        del packed
    else:
        new_id = degree_order_share(edges, scale, world, device) if reorder else None
        G._mark("deal_ids")
        s, d = shuffle_edges(edges, new_id, n_vertices, world)
    use_native = (torch.device(device).type == "cuda") if native is None else native
    if use_native:
        ng = G.build_native([(s, d)], n_vertices, rank, world, None, bin_width=bin_width, tile=tile,
                            keep_keys=keep_keys)
        ng.new_id = new_id
        return ng
    sl = G.vertex_slices(n_vertices, world)
    v_lo, v_hi = rank * sl, min(n_vertices, (rank + 1) * sl)
    shard = G.merge_shards([(s, d - v_lo)], v_lo, v_hi, n_vertices, sl)
    shard.new_id = new_id
    return shard


def rmat_shard(scale: int, edge_factor: int, rank: int, world: int, device, seed: int = 1,
               chunk: int = 1 << 26, reorder: bool = True):
    """Generate the global R-MAT stream, keep this rank's destinations.

    reorder=True relabels vertices by descending out-degree (see degree_order);
    PageRank values are invariant to the relabeling (map back with the returned
    ``new_id`` if original ids are needed).
    """
    edges, n_edges = rmat_input(scale, edge_factor, device, seed, chunk)
    shard = build_rmat_shard(edges, scale, rank, world, device, reorder=reorder, seed=seed)
    return shard, n_edges


def main(argv=None):
    ap = common_parser("Distributed PageRank (MI355X-native)")
    ap.add_argument("--n-iterations", type=int, default=10)
    ap.add_argument("--q", type=float, default=0.15)
    ap.add_argument("--semantics", choices=["reference", "standard"], default="reference")
    ap.add_argument("--edges", default=None, help="whitespace-separated 'src dst' edge file")
    ap.add_argument("--rmat-scale", type=int, default=None, help="synthetic Graph500 R-MAT graph")
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--top", type=int, default=20, help="print only the top ranks of large graphs")
    ap.add_argument("--spmv", choices=["blocked", "pull"], default=None,
                    help="SpMV form (default: blocked K4b on GPUs, pull on the CPU)")
    ap.add_argument("--exchange", choices=["ghost", "allgather"], default="ghost")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="ghost exchange under the own-source SpMV")
    add_ckpt_args(ap)
    a = ap.parse_args(argv)
    rt = init_from_args(a, "PageRank")
    ids = None
    if a.rmat_scale:
        shard, _ = rmat_shard(a.rmat_scale, a.edge_factor, rt.rank, rt.world_size, rt.device, a.seed + 1)
    else:
        if a.edges:
            src, dst = load_edges(a.edges)
        else:
            src = torch.tensor([e[0] for e in TOY_EDGES], dtype=torch.int32)
            dst = torch.tensor([e[1] for e in TOY_EDGES], dtype=torch.int32)
        s, d, ids = compact_ids(src.long(), dst.long())
        shard = G.build_shard(s.to(torch.int32).to(rt.device), d.to(torch.int32).to(rt.device),
                              len(ids), rt.rank, rt.world_size)
    pr = PageRank(PageRankConfig(q=a.q, n_iterations=a.n_iterations, semantics=a.semantics,
                                 spmv=a.spmv or "", exchange=a.exchange, overlap=a.overlap),
                  shard, rt.world_size)
    if a.resume and a.ckpt_dir:
        sd = checkpoint.load(a.ckpt_dir, "pagerank_state", rt.rank, per_rank=True)
        if sd is not None:
            pr.load_state_dict(sd)
            rt.log(f"Resumed from iteration {pr.t}")
    sink = obs.MetricsSink(a.metrics_out, rt.rank)
    if sink.enabled or obs.roctx_enabled():
        pr.timer = obs.PhaseTimer(rt.device)
    while pr.t < a.n_iterations:
        pr.step()
        sink.log(phases=pr.timer.take() if pr.timer else None, iteration=pr.t,
                 bytes_exchanged=getattr(pr, "bytes_exchanged", 0), world_size=rt.world_size,
                 exchange=pr.exchange)
        if a.ckpt_dir and a.ckpt_every and pr.t % a.ckpt_every == 0:
            checkpoint.save(pr.state_dict(), a.ckpt_dir, "pagerank_state", rt.rank, per_rank=True)
    if a.ckpt_dir:
        checkpoint.save(pr.state_dict(), a.ckpt_dir, "pagerank_state", rt.rank, per_rank=True)
    ranks = pr.collect()
    if shard.new_id is not None:
        # report the R-MAT generator's own vertex ids (the degree relabeling depends on W)
        inv = torch.empty_like(shard.new_id, dtype=torch.int64)
        inv[shard.new_id.long()] = torch.arange(shard.new_id.numel(), device=inv.device)
        inv = inv.cpu()
        ranks = {int(inv[v]): r for v, r in ranks.items()}
    if rt.is_main:
        items = list(ranks.items())
        if ids is None and len(items) > a.top:
            items = sorted(items, key=lambda kv: -kv[1])[: a.top]
        for v, r in items:
            vid = int(ids[v]) if ids is not None else v
            print("%s has rank: %s." % (vid, r))
    sink.close()
    runtime.shutdown()
    return ranks if ids is None else {int(ids[v]): r for v, r in ranks.items()}
