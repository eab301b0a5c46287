"""Native PageRank adjacency build (csrc/kernels/graph_build.hip, dalgo.ops.graph.build_native)
against the torch path: same distinct edge set per rank, the K4b layout's SpMV equals the
pull SpMV over the same edges, whole PageRank runs equal the torch-built model."""
import pytest
import torch

from dalgo.apps.pagerank_app import build_rmat_native, build_rmat_shard, rmat_input
from dalgo.models.pagerank import PageRank, PageRankConfig
from dalgo.ops import graph as G

pytestmark = pytest.mark.gpu


def _edge_set(shard):
    E = shard.n_edges
    return (shard.dstl[:E].long() << 32) | shard.src[:E].long()


@pytest.mark.parametrize("reorder", [True, False])
def test_degree_count_matches_bincount(cuda, reorder):
    s, _ = G.rmat_edges(1 << 20, 16, seed=3, device=cuda)
    deg = torch.zeros(1 << 16, dtype=torch.int32, device=cuda)
    G.degree_count_(deg, s)
    G.degree_count_(deg, s[: 1000])
    ref = torch.bincount(s.long(), minlength=1 << 16) + torch.bincount(s[:1000].long(), minlength=1 << 16)
    assert torch.equal(deg.long(), ref)


@pytest.mark.parametrize("lo_bits", [13, 5])
def test_run_sort_completes_high_bit_sort(cuda, lo_bits):
    """gb_sort over the bits above lo_bits + gb_run_sort (each run of equal high bits sorted
    on its low bits in place) == a full sort: runs of 1, 2-64 (per-key ranks), 65-256 (wave
    network), 257-70000 keys (block counting sort, copies kept), runs crossing 2048-key
    tiles."""
    g = torch.Generator().manual_seed(11)
    parts = [torch.randint(0, 1 << 20, (300_000,), generator=g)]          # mostly runs of 1
    parts.append(torch.randint(0, 1 << 14, (200_000,), generator=g))      # runs of ~12
    for ln, hv in ((17, 1 << 21), (40, (1 << 21) + 1), (300, (1 << 21) + 2), (5000, (1 << 21) + 3),
                   (70000, (1 << 21) + 4), (256, (1 << 21) + 5), (257, (1 << 21) + 6),
                   (100, (1 << 21) + 7), (64, (1 << 21) + 8), (65, (1 << 21) + 9)):
        parts.append(torch.full((ln,), hv))
    hi = torch.cat(parts).to(torch.int64)
    lo = torch.randint(0, 1 << lo_bits, (hi.numel(),), generator=g)
    keys = ((hi << lo_bits) | lo)[torch.randperm(hi.numel(), generator=g)].to(cuda)
    n = keys.numel() - 7                                                  # a ragged end
    out = torch.empty_like(keys)
    ops = G._ext.ops()
    ops.gb_sort(keys, n, 21 + 1 + lo_bits, out, lo_bits)
    cnt = ops.gb_run_sort(out, n, lo_bits).tolist()
    assert cnt[0] >= 4                                                    # block tier ran
    assert torch.equal(out[:n].cpu(), torch.sort(keys[:n].cpu()).values)


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("reorder", [True, False])
def test_native_edges_equal_torch_shard(cuda, world, reorder):
    """Every rank's distinct edges (global ids) == the torch-built (dst, src) shard, and the
    out-degree of every local source counts exactly its distinct out-edges."""
    scale = 14
    edges, _ = rmat_input(scale, 8, torch.device(cuda), seed=5, chunk=1 << 15)
    for rank in range(world):
        if reorder and world > 1:
            # the relabeling needs every rank's degree share (a collective): one process
            # emulates it with the full count
            new_id = _full_order(edges, scale, world, cuda)
            ng = G.build_native(edges, 1 << scale, rank, world, new_id, keep_keys=True)
            ref = _torch_shard(edges, scale, rank, world, new_id)
        else:
            ng = build_rmat_native(edges, scale, rank, world, cuda, reorder=reorder, keep_keys=True)
            ref = build_rmat_shard(edges, scale, rank, world, cuda, reorder=reorder)
        sh = ng.to_shard()
        assert ng.n_edges == ref.n_edges
        assert torch.equal(_edge_set(sh), _edge_set(ref))
        # distinct out-degree per local source
        sl = ng.slice_size
        src = ref.src[: ref.n_edges].long()
        own = (src >= ng.v_lo) & (src < ng.v_hi)
        od = torch.zeros_like(ng.outdeg_loc, dtype=torch.int64)
        od.index_add_(0, src[own] - ng.v_lo, torch.ones_like(src[own]))
        if ng.ghosts is not None and ng.n_ghost:
            gi = torch.searchsorted(ng.ghosts, src[~own])
            od.index_add_(0, sl + gi, torch.ones_like(gi))
        assert torch.equal(od, ng.outdeg_loc.long())


def _full_order(edges, scale, world, cuda):
    from dalgo.apps.pagerank_app import deal_ids
    n = 1 << scale
    deg = torch.zeros(n, dtype=torch.int32, device=cuda)
    for s, _ in edges:
        G.degree_count_(deg, s)
    order = torch.argsort(-deg.long() * n - torch.arange(n, device=cuda))
    return deal_ids(order, n, world).to(torch.int32)


def _torch_shard(edges, scale, rank, world, new_id):
    n = 1 << scale
    sl = G.vertex_slices(n, world)
    v_lo, v_hi = rank * sl, min(n, (rank + 1) * sl)
    parts = []
    for s, d in edges:
        s, d = new_id[s.long()], new_id[d.long()]
        keep = (d >= v_lo) & (d < v_hi)
        parts.append((s[keep], d[keep] - v_lo))
    return G.merge_shards(parts, v_lo, v_hi, n, sl)


@pytest.mark.parametrize("world", [1, 2])
def test_native_layout_spmv_matches_pull(cuda, world):
    """K4b over the native layout (local [own | ghost] source space) == the pull SpMV over
    the same edges, per rank, on random contributions (some absent)."""
    scale = 15
    edges, _ = rmat_input(scale, 16, torch.device(cuda), seed=9, chunk=1 << 16)
    g = torch.Generator(device="cpu").manual_seed(1)
    for rank in range(world):
        ng = build_rmat_native(edges, scale, rank, world, cuda, reorder=False, keep_keys=True)
        sl = ng.slice_size
        nc = sl + ng.n_ghost
        c = torch.rand(nc, generator=g).to(cuda)
        c[torch.rand(nc, generator=g).to(cuda) < 0.2] = -1.0
        lay = ng.layout
        acc = torch.empty(ng.n_local, device=cuda)
        pres = torch.empty(ng.n_local, dtype=torch.int32, device=cuda)
        G.pb_spmv(lay, c, acc, pres)
        # pull reference in the same local source space
        sh = ng.to_shard()
        gs = sh.src[: sh.n_edges].long()
        d = sh.dstl[: sh.n_edges].long()
        own = (gs >= ng.v_lo) & (gs < ng.v_hi)
        li = torch.where(own, gs - ng.v_lo, torch.zeros_like(gs))
        if ng.ghosts is not None and ng.n_ghost:
            li = torch.where(own, li, sl + torch.searchsorted(ng.ghosts, gs))
        cv = c[li].double()
        ref = torch.zeros(ng.n_local, dtype=torch.float64, device=cuda)
        ref.index_add_(0, d, cv.clamp_min(0))
        hit = torch.zeros(ng.n_local, dtype=torch.int64, device=cuda)
        hit.index_add_(0, d, (cv >= 0).long())
        assert torch.equal(pres.bool(), hit > 0)
        assert torch.allclose(acc.double(), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("sem", ["reference", "standard"])
def test_native_pagerank_equals_torch_build(cuda, sem):
    scale = 16
    edges, _ = rmat_input(scale, 16, torch.device(cuda), seed=2, chunk=1 << 18)
    ng = build_rmat_native(edges, scale, 0, 1, cuda, reorder=True)
    sh = build_rmat_shard(edges, scale, 0, 1, cuda, reorder=True)
    a = PageRank(PageRankConfig(semantics=sem, spmv="blocked"), ng).fit()
    b = PageRank(PageRankConfig(semantics=sem, spmv="pull"), sh).fit()
    assert a.N == b.N
    assert torch.equal(a.r >= 0, b.r >= 0)
    assert torch.allclose(a.r, b.r, rtol=2e-5, atol=1e-12)


def test_rank_by_degree_matches_argsort(cuda):
    from dalgo.apps.pagerank_app import rank_by_degree
    g = torch.Generator().manual_seed(4)
    deg = torch.randint(0, 50, (100_003,), generator=g, dtype=torch.int32)
    ref = rank_by_degree(deg)
    got = rank_by_degree(deg.to(cuda)).cpu()
    assert torch.equal(got, ref)


def test_degree_sorted_matches_bincount(cuda):
    s, _ = G.rmat_edges(3 << 20, 18, seed=7, device=cuda)
    deg = torch.full((1 << 18,), 5, dtype=torch.int32, device=cuda)
    G.degree_sorted_(deg, s, 18)
    ref = torch.bincount(s.long(), minlength=1 << 18) + 5
    assert torch.equal(deg.long(), ref)


@pytest.mark.parametrize("world", [1, 3])
def test_cell_matrix_layout_equals_entry_scan(cuda, world, monkeypatch):
    """The (block, bin) cell-matrix path of the run / tile tables (gb_cell_* kernels) and
    the per-entry flag + scan + run-sort fallback build the same K4b layout, field by
    field, on every rank (ghost blocks included)."""
    scale = 15
    edges, _ = rmat_input(scale, 16, torch.device(cuda), seed=21, chunk=1 << 16)
    fields = ("srcl", "tile_e", "tile_ent", "tile_run", "chunk_tile", "wu_tile", "wu_chunk", "chunk_slo",
              "chunk_ns", "chunk_run", "run_delta", "dloc", "wi_bin", "wi_lo", "wi_slab", "split_bin",
              "split_first", "split_count")
    for rank in range(world):
        a = build_rmat_native(edges, scale, rank, world, cuda, reorder=False, bin_width=8192, tile=2048).layout
        monkeypatch.setattr(G, "CELL_CAP", 0)
        b = build_rmat_native(edges, scale, rank, world, cuda, reorder=False, bin_width=8192, tile=2048).layout
        monkeypatch.undo()
        for f in fields:
            assert torch.equal(getattr(a, f), getattr(b, f)), f
        for f in ("n_chunks", "n_entries", "n_src", "max_runs", "n_local"):
            assert getattr(a, f) == getattr(b, f), f


def test_native_relabel_many_buckets_equals_torch_shard(cuda):
    """The one-rank packed path with degree relabeling at scale 20: 128 source buckets of
    the bucketed relabel (gb_relabel_bucket_kernel, one block per bucket) -- enough blocks
    in flight for a cross-block race on the edge words to show. Edge set, edge count and the
    distinct out-degree of every source equal the torch build."""
    scale = 20
    edges, _ = rmat_input(scale, 16, torch.device(cuda), seed=13, chunk=1 << 22)
    ng = build_rmat_native(edges, scale, 0, 1, cuda, reorder=True, keep_keys=True)
    ref = build_rmat_shard(edges, scale, 0, 1, cuda, reorder=True)
    assert torch.equal(ng.new_id.long(), ref.new_id.long())
    assert ng.n_edges == ref.n_edges
    sh = ng.to_shard()
    assert torch.equal(_edge_set(sh), _edge_set(ref))
    od = torch.bincount(ref.src[: ref.n_edges].long(), minlength=ng.outdeg_loc.numel())
    assert torch.equal(od, ng.outdeg_loc.long())
    # the relabel is a bijection and the raw distinct count is preserved by it
    raw = torch.unique(torch.cat([(s.long() << 32) | d.long() for s, d in edges]))
    assert int(raw.numel()) == ng.n_edges


@pytest.mark.parametrize("world", [1, 3, 8])
def test_owner_partition_matches_torch(cuda, world):
    """gb_owner_partition (relabel + group by destination owner) == the torch path: the same
    per-owner counts and, per owner, the same multiset of packed edges."""
    scale = 16
    s, d = G.rmat_edges((1 << 20) + 3, scale, seed=17, device=cuda)        # ragged length
    new_id = torch.randperm(1 << scale, device=cuda).to(torch.int32)
    got, cg = G.owner_partition(s, d, new_id, 1 << scale, world)
    exp, ce = G.owner_partition(s.cpu(), d.cpu(), new_id.cpu(), 1 << scale, world)
    assert cg == ce and sum(cg) == s.numel()
    a = 0
    for c in cg:
        assert torch.equal(torch.sort(got[a:a + c].cpu()).values, torch.sort(exp[a:a + c]).values)
        a += c


@pytest.mark.parametrize("world", [1, 3, 8])
def test_bucketed_owner_partition_matches_torch(cuda, world):
    """build_rmat_sharded's GPU shuffle source: source partition + degrees, bucketed source
    relabel, destination-bit partition, then the owner pass relabelling destinations in
    place (gb_owner_partition_packed) == the torch owner partition of the raw edges."""
    scale = 17
    s, d = G.rmat_edges((1 << 20) + 5, scale, seed=19, device=cuda)
    new_id = torch.randperm(1 << scale, device=cuda).to(torch.int32)
    packed, deg = G.partition_edges([(s, d)], scale)
    assert torch.equal(deg.long().cpu(), torch.bincount(s.long().cpu(), minlength=1 << scale))
    packed = G.relabel_partition_dst(packed, new_id, scale)
    got, cg = G.owner_partition_packed(packed, new_id, 1 << scale, world)
    exp, ce = G.owner_partition(s.cpu(), d.cpu(), new_id.cpu(), 1 << scale, world)
    assert cg == ce and sum(cg) == s.numel()
    a = 0
    for c in cg:
        assert torch.equal(torch.sort(got[a:a + c].cpu()).values, torch.sort(exp[a:a + c]).values)
        a += c


@pytest.mark.parametrize("world", [2, 8])
def test_deal_kernel_matches_torch(cuda, world):
    from dalgo.apps.pagerank_app import deal_ids
    n = 1 << 16
    order = torch.randperm(n)
    exp = deal_ids(order, n, world)
    got = deal_ids(order.to(cuda), n, world)
    assert torch.equal(got.long().cpu(), exp.long())


@pytest.mark.parametrize("world,hubs", [(1, 0), (1, 300), (2, 300), (8, 0), (8, 300)])
def test_degree_new_id_matches_torch(cuda, world, hubs):
    """The fused ranking (gb_rank_keys + sort + masked gb_deal) == deal_ids(rank_by_degree)
    on the CPU: degree ties (small degree range) broken by descending id, snake deal; hubs
    with degrees past 16 bits (ties among them too)."""
    from dalgo.apps.pagerank_app import deal_ids, degree_new_id, rank_by_degree
    n = 1 << 17
    g = torch.Generator().manual_seed(6)
    deg = torch.randint(0, 40, (n,), generator=g, dtype=torch.int32)
    if hubs:
        idx = torch.randperm(n, generator=g)[:hubs]
        deg[idx] = torch.randint(1 << 16, (1 << 16) + 50, (hubs,), generator=g, dtype=torch.int32)
    exp = deal_ids(rank_by_degree(deg), n, world).to(torch.int32)
    got = degree_new_id(deg.to(cuda), n, world).cpu()
    assert got.dtype == torch.int32 and torch.equal(got, exp)


def test_bitmap_ghost_ids(cuda):
    g = torch.Generator().manual_seed(5)
    bm = torch.randint(-(1 << 31), (1 << 31) - 1, (5000,), generator=g, dtype=torch.int64).to(torch.int32)
    bm[::7] = 0
    bits = (bm.long()[:, None] >> torch.arange(32)) & 1
    exp = torch.nonzero(bits.flatten()).flatten()
    pc = bits.sum(1)
    prefix = (torch.cumsum(pc, 0) - pc).to(cuda)
    out = torch.empty(exp.numel(), dtype=torch.int64, device=cuda)
    G._ext.ops().gb_bitmap_ids(bm.to(cuda), prefix, out)
    assert torch.equal(out.cpu(), exp)
