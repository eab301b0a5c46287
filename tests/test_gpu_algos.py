"""GPU numerics of K2/K3 (k-means), K4 (PageRank), K5 (ALS), K9 (closure) and the
end-to-end models against the torch-CPU references."""
import math

import numpy as np
import pytest
import torch

from dalgo.ops import graph as G
from dalgo.ops import kmeans as K

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ k-means
# bf16 with DP 64 / 128 takes the pipelined MFMA form (ragged tile groups, one and many
# 128-centre chunks); f32 and small d the generic form
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("d,k,n", [(2, 2, 6), (16, 40, 3000), (50, 33, 4099), (64, 128, 513),
                                   (100, 1500, 9000), (128, 600, 70001), (128, 1024, 20000),
                                   (128, 4096, 20000)])
def test_kmeans_assign_matches_reference(cuda, dtype, d, k, n):
    _check_assign(cuda, dtype, d, k, n)


@pytest.mark.parametrize("d", [8, 128])
def test_kmeans_assign_ties(cuda, d):
    """Exact ties resolve to the lowest id across sub-tiles, chunks and lane halves."""
    X = torch.zeros(300, d)
    C0 = torch.zeros(1100, d) + 50.0
    for c in (3, 7, 12, 515, 1030):
        C0[c] = 0.0
        C0[c, c % d] = 1.0
    a = K.assign(K.prepare_points(X.to(cuda).bfloat16()), K.make_centers(C0, torch.bfloat16, cuda)).cpu()
    assert a.tolist() == [3] * 300


def _check_assign(cuda, dtype, d, k, n):
    g = torch.Generator().manual_seed(d + k)
    X = (torch.randn(n, d, generator=g) * 3).to(dtype)
    C0 = torch.randn(k, d, generator=g) * 3
    Xc = K.prepare_points(X)
    cen_c = K.make_centers(C0, dtype, "cpu")
    a_ref = K.assign(Xc, cen_c)
    Xd = K.prepare_points(X.to(cuda))
    cen_d = K.make_centers(C0, dtype, cuda)
    mind = torch.empty(n, device=cuda)
    sse = torch.zeros(1, dtype=torch.float64, device=cuda)
    a = K.assign(Xd, cen_d, mind=mind, sse=sse).cpu()
    # scores computed in f32 on the GPU vs f64 on the CPU: allow rare near-ties
    agree = (a == a_ref).float().mean().item()
    assert agree > 0.999, agree
    # where they differ the two distances must be (nearly) equal
    Xf = Xc.double()
    Cr = cen_c.Cq[:k, :d].double()
    dist = torch.cdist(Xf, Cr) ** 2
    dd = dist.gather(1, a.long()[:, None]) - dist.gather(1, a_ref.long()[:, None])
    assert dd.abs().max().item() < 1e-3 * (1 + dist.max().item())
    assert torch.allclose(mind.cpu().double(), dist.gather(1, a.long()[:, None])[:, 0],
                          rtol=1e-3, atol=1e-2)
    assert float(sse.item()) == pytest.approx(float(mind.double().sum().item()), rel=1e-6)


def test_kmeans_ties_lowest_index(cuda):
    X = torch.tensor([[0.0, 0.0]] * 5)
    C0 = torch.tensor([[1.0, 0.0], [-1.0, 0.0], [0.0, 1.0]])   # all equidistant
    a = K.assign(K.prepare_points(X.to(cuda)), K.make_centers(C0, torch.float32, cuda)).cpu()
    assert a.tolist() == [0] * 5


@pytest.mark.parametrize("k,skew", [(1024, "uniform"), (1500, "uniform"), (2048, "uniform"),
                                    (2048, "one-cluster"), (1500, "two-clusters"),
                                    (3000, "uniform"), (16384, "uniform")])
def test_kmeans_sorted_accumulate(cuda, k, skew):
    """K3 sorted accumulate: the coalesced chunked scatter (k <= 2048) and the per-row
    LDS-cursor scatter (k > 2048): several blocks, full and partial 32K-row chunks; exact
    counts, f64-checked sums. k = 1500 / 2048 run the two-clusters-per-thread scan of the
    chunked scatter (kScKmax boundary); "one-cluster" puts every row of a 32K chunk in one
    cluster (15-bit local rank at its limit); k = 16384 needs the > 64 KB dynamic-LDS scan."""
    n, d = 300_001, 64
    g = torch.Generator().manual_seed(3)
    X = torch.randn(n, d, generator=g).to(torch.bfloat16)
    if skew == "one-cluster":
        a = torch.full((n,), k - 1, dtype=torch.int32)
    elif skew == "two-clusters":
        a = torch.where(torch.rand(n, generator=g) < 0.5, 7, k - 2).to(torch.int32)
    else:
        a = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    DP = K.kmeans_dp(d)
    S = torch.zeros(k, DP, device=cuda)
    cnt = torch.zeros(k, dtype=torch.int64, device=cuda)
    K.accumulate(K.prepare_points(X.to(cuda)), a.to(cuda), k, DP, S, cnt)
    Sr = torch.zeros(k, DP, dtype=torch.float64)
    Sr[:, :d].index_add_(0, a.long(), X.double())
    assert torch.equal(cnt.cpu(), torch.bincount(a.long(), minlength=k))
    assert torch.allclose(S.cpu().double(), Sr, atol=1e-2, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_kmeans_accumulate_update(cuda, dtype):
    n, d, k = 50_000, 100, 70
    g = torch.Generator().manual_seed(1)
    X = torch.randn(n, d, generator=g).to(dtype)
    a = torch.randint(0, k - 3, (n,), generator=g, dtype=torch.int32)   # last 3 clusters empty
    DP = K.kmeans_dp(d)
    S = torch.zeros(k, DP, device=cuda)
    cnt = torch.zeros(k, dtype=torch.int64, device=cuda)
    K.accumulate(K.prepare_points(X.to(cuda)), a.to(cuda), k, DP, S, cnt)
    Sr = torch.zeros(k, DP, dtype=torch.float64)
    Sr[:, :d].index_add_(0, a.long(), X.double())
    cr = torch.bincount(a.long(), minlength=k)
    assert torch.equal(cnt.cpu(), cr)
    assert torch.allclose(S.cpu().double(), Sr, atol=1e-2, rtol=1e-4)
    C0 = torch.randn(k, d, generator=g)
    cen = K.make_centers(C0, dtype, cuda)
    sh = torch.zeros(1, device=cuda)
    K.update(cen, S, cnt, sh)
    exp = torch.where(cr[:, None] > 0, Sr[:, :d] / cr.clamp_min(1)[:, None].double(), C0.double())
    assert torch.allclose(cen.C.cpu().double(), exp, atol=1e-4)
    assert torch.equal(cen.C[-3:].cpu(), C0[-3:])   # empty clusters keep the stale centre
    rq = cen.Cq[:k, :d].float()
    assert torch.allclose(cen.hn[:k], 0.5 * (rq * rq).sum(1), rtol=1e-5)
    assert (cen.hn[k:] > 1e29).all()


def test_kmeans_model_gpu_vs_cpu(cuda):
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    X = blobs(20_000, 16, 8, seed=5)
    cfg = KMeansConfig(k=8, n_iterations=6, seed=3)
    kc = KMeans(cfg, X, 0, X.shape[0])
    kc.fit()
    kg = KMeans(cfg, X.to(cuda), 0, X.shape[0])
    kg.fit()
    assert torch.allclose(kg.centers.cpu(), kc.centers, atol=1e-3)
    assert kg.history.sse[-1] == pytest.approx(kc.history.sse[-1], rel=1e-4)


def test_kmeans_toy_gpu(cuda):
    from dalgo.models.kmeans import KMeans, KMeansConfig
    X = torch.tensor([[1, 2], [1, 4], [1, 0], [10, 2], [10, 4], [10, 0]], dtype=torch.float32)
    km = KMeans(KMeansConfig(k=2), X.to(cuda), 0, 6,
                init_centers=torch.tensor([[1.0, 4.0], [10.0, 0.0]]))
    km.fit()
    assert km.centers.cpu().tolist() == [[1.0, 2.0], [10.0, 2.0]]


# ------------------------------------------------------------------ PageRank
def test_rmat_generator_matches_cpu(cuda):
    s, d = G.rmat_edges(5000, 14, seed=11, e_off=123, device=cuda)
    sc, dc = G.rmat_edges(5000, 14, seed=11, e_off=123)
    assert torch.equal(s.cpu(), sc) and torch.equal(d.cpu(), dc)
    assert int(s.max()) < (1 << 14) and int(s.min()) >= 0


@pytest.mark.parametrize("frac_absent", [0.0, 0.3])
def test_pr_spmv_matches_reference(cuda, frac_absent):
    nv = 1 << 13
    s, d = G.rmat_edges(200_000, 13, seed=3)
    sh_c = G.build_shard(s, d, nv, 0, 1)
    sh_d = G.build_shard(s.to(cuda), d.to(cuda), nv, 0, 1)
    g = torch.Generator().manual_seed(0)
    c = torch.rand(nv, generator=g)
    c[torch.rand(nv, generator=g) < frac_absent] = -1.0
    acc_c = torch.zeros(nv, dtype=torch.float64)
    pres_c = torch.zeros(nv, dtype=torch.int32)
    G.pr_spmv(sh_c, c.double(), acc_c, pres_c)
    acc = torch.zeros(nv, device=cuda)
    pres = torch.zeros(nv, dtype=torch.int32, device=cuda)
    G.pr_spmv(sh_d, c.to(cuda), acc, pres)
    assert torch.equal(pres.cpu(), pres_c)
    assert torch.allclose(acc.cpu().double(), acc_c, rtol=1e-5, atol=1e-5)
    # two passes over a source split of the same edges (the overlapped ghost exchange:
    # own-slice sources, then the accumulate pass over the rest) == one pass
    E = sh_d.n_edges
    m = sh_d.src[:E] < nv // 3

    def part(mask):
        k = int(mask.sum().item())
        kp = (k + 3) // 4 * 4
        s_ = torch.full((kp,), -1, dtype=torch.int32, device=cuda)
        d_ = torch.full((kp,), -1, dtype=torch.int32, device=cuda)
        s_[:k] = sh_d.src[:E][mask]
        d_[:k] = sh_d.dstl[:E][mask]
        return G.GraphShard(s_, d_, k, sh_d.v_lo, sh_d.v_hi, sh_d.n_vertices, sh_d.slice_size)

    acc2 = torch.zeros(nv, device=cuda)
    pres2 = torch.zeros(nv, dtype=torch.int32, device=cuda)
    G.pr_spmv(part(m), c.to(cuda), acc2, pres2)
    G.pr_spmv(part(~m), c.to(cuda), acc2, pres2, accumulate=True)
    assert torch.equal(pres2.cpu(), pres_c)
    assert torch.allclose(acc2.cpu().double(), acc_c, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("sem", ["reference", "standard"])
def test_pagerank_gpu_vs_cpu(cuda, sem):
    from dalgo.models.pagerank import PageRank, PageRankConfig
    s, d = G.rmat_edges(100_000, 12, seed=8)
    nv = 1 << 12
    rc = PageRank(PageRankConfig(semantics=sem), G.build_shard(s, d, nv, 0, 1)).fit().collect()
    rg = PageRank(PageRankConfig(semantics=sem),
                  G.build_shard(s.to(cuda), d.to(cuda), nv, 0, 1)).fit().collect()
    assert set(rc) == set(rg)
    assert max(abs(rc[v] - rg[v]) for v in rc) < 1e-6


def test_pagerank_toy_gpu(cuda):
    from dalgo.models.pagerank import PageRank, PageRankConfig
    src = torch.tensor([1, 1, 2, 3], dtype=torch.int32, device=cuda)
    dst = torch.tensor([2, 3, 3, 1], dtype=torch.int32, device=cuda)
    r = PageRank(PageRankConfig(), G.build_shard(src, dst, 4, 0, 1)).fit().collect()
    assert r[1] == pytest.approx(0.38891305880091237, abs=1e-6)
    assert r[2] == pytest.approx(0.214416470596171, abs=1e-6)
    assert r[3] == pytest.approx(0.3966704706029163, abs=1e-6)


@pytest.mark.parametrize("bw,chunk,tile,min_piece", [(16384, 1 << 17, 4096, 1 << 14),
                                                     (8192, 4096, 100, 64)])
def test_pb_spmv_matches_pull(cuda, bw, chunk, tile, min_piece):
    """K4b two-level propagation-blocked SpMV == pull SpMV (acc to f32 summation order, pres
    exact): many chunks and tiles, entries pre-combined per chunk, split bins (slabs), absent
    sources, 1 and 3 destination slices."""
    from dalgo.ops import graph as G
    g = torch.Generator().manual_seed(5)
    n, E = 100_000, 2_000_000
    # skewed sources and destinations: hot destinations repeat inside a chunk
    src = (torch.rand(E, generator=g) ** 2 * n).to(torch.int32)
    dst = (torch.rand(E, generator=g) ** 3 * n).to(torch.int32)
    for W, r in ((1, 0), (3, 1)):
        sh = G.build_shard(src.to(cuda), dst.to(cuda), n, r, W)
        lay = G.build_blocked(sh, bw, chunk, tile, min_piece=min_piece)
        assert lay.n_entries < sh.n_edges            # hot destinations pre-combined
        if min_piece < 1000:
            assert lay.split_bin.numel() > 0         # slab path exercised
        c = (torch.rand(n, generator=g) * 2 - 0.5).to(cuda)   # negatives = absent vertices
        a1 = torch.zeros(sh.n_local, device=cuda)
        p1 = torch.zeros(sh.n_local, dtype=torch.int32, device=cuda)
        a2, p2 = torch.zeros_like(a1), torch.zeros_like(p1)
        G.pr_spmv(sh, c, a1, p1)
        for _ in range(2):                           # val / slabs are reused across calls
            a2.zero_(); p2.zero_()
            G.pb_spmv(lay, c, a2, p2)
        torch.cuda.synchronize()
        assert torch.equal(p1, p2)
        assert torch.allclose(a1, a2, rtol=1e-5, atol=1e-4)
        # f64 reference
        cc = c.double().cpu()
        s64 = sh.src[:sh.n_edges].long().cpu()
        d64 = sh.dstl[:sh.n_edges].long().cpu()
        ref = torch.zeros(sh.n_local, dtype=torch.float64).index_add_(0, d64, cc[s64].clamp_min(0))
        # exact u64 fixed-point sums rounded once: f32 rounding of the exact sum
        assert torch.allclose(a2.double().cpu(), ref, rtol=2e-7, atol=1e-12)


def test_pb_spmv_empty_shard_writes_zeros(cuda):
    """A rank whose slice has no in-edges: every output is still written (no pre-zeroing)."""
    from dalgo.ops import graph as G
    src = torch.tensor([0, 1], dtype=torch.int32, device=cuda)
    dst = torch.tensor([1, 0], dtype=torch.int32, device=cuda)
    sh = G.build_shard(src, dst, 40000, 1, 2)
    assert sh.n_edges == 0
    lay = G.build_blocked(sh)
    acc = torch.full((sh.n_local,), 5.0, device=cuda)
    pres = torch.ones(sh.n_local, dtype=torch.int32, device=cuda)
    G.pb_spmv(lay, torch.rand(40000, device=cuda), acc, pres)
    torch.cuda.synchronize()
    assert float(acc.abs().max()) == 0.0 and int(pres.max()) == 0


def test_pb_spmv_fixed_point_scale_follows_data(cuda):
    """PageRank-sized contributions (~1e-9) into hub destinations: the u64 fixed-point scale
    comes from the data (sum of the present c), so the sums keep ~f32 accuracy relative to
    an f64 reference (a worst-case in-degree x c_max scale left ~1e-4 here)."""
    from dalgo.ops import graph as G
    g = torch.Generator().manual_seed(7)
    n, E = 1 << 20, 8_000_000
    src = torch.randint(0, n, (E,), generator=g, dtype=torch.int32)
    dst = (torch.rand(E, generator=g) ** 4 * n).to(torch.int32)          # hubs near 0
    sh = G.build_shard(src.to(cuda), dst.to(cuda), n, 0, 1)
    lay = G.build_blocked(sh)
    c = (torch.rand(n, generator=g) * 2e-9).to(cuda)
    acc = torch.zeros(sh.n_local, device=cuda)
    pres = torch.zeros(sh.n_local, dtype=torch.int32, device=cuda)
    G.pb_spmv(lay, c, acc, pres)
    torch.cuda.synchronize()
    s64 = sh.src[:sh.n_edges].long().cpu()
    d64 = sh.dstl[:sh.n_edges].long().cpu()
    ref = torch.zeros(sh.n_local, dtype=torch.float64).index_add_(0, d64, c.double().cpu()[s64])
    assert torch.allclose(acc.double().cpu(), ref, rtol=3e-7, atol=1e-20)


def test_pb_spmv_split_phases_bitwise_equal(cuda):
    """Phase 1 split at the own-slice / ghost source boundary (the overlapped exchange's
    call sequence) gives bitwise the same result as one call: the u64 fixed-point sums do
    not depend on the order of the adds."""
    from dalgo.ops import graph as G
    g = torch.Generator().manual_seed(3)
    n, E, split = 200_000, 3_000_000, 70_000
    src = (torch.rand(E, generator=g) ** 2 * n).to(torch.int32)
    dst = torch.randint(0, 100_000, (E,), generator=g, dtype=torch.int32)
    sh = G.build_shard(src.to(cuda), dst.to(cuda), 100_000, 0, 1)
    lay = G.build_blocked(sh, src_split=split)
    nb = lay.n_wu_below
    assert 0 < nb < lay.wu_chunk.numel()
    slo = lay.chunk_slo.long()
    wc = lay.wu_chunk.long()
    assert bool((slo[wc[:nb]] < split).all()) and bool((slo[wc[nb:]] >= split).all())
    c = torch.rand(n, generator=g).to(cuda)
    a1 = torch.zeros(sh.n_local, device=cuda)
    p1 = torch.zeros(sh.n_local, dtype=torch.int32, device=cuda)
    a2, p2 = torch.zeros_like(a1), torch.zeros_like(p1)
    G.pb_spmv(lay, c, a1, p1)
    G.pb_spmv(lay, c, a2, p2, wu_range=(0, nb), phases=1)
    G.pb_spmv(lay, c, a2, p2, wu_range=(nb, 1 << 31), phases=1)
    G.pb_spmv(lay, c, a2, p2, phases=2)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2) and torch.equal(p1, p2)


def test_pb_spmv_many_runs_global_delta_path(cuda):
    """A chunk whose edges reach more than 4096 destination bins: phase 1 reads its run
    deltas from global memory instead of the LDS table (the large-slice form)."""
    from dalgo.ops import graph as G
    g = torch.Generator().manual_seed(11)
    n, E = 5000 * 8192, 200_000
    src = torch.randint(0, 8192, (E,), generator=g, dtype=torch.int32)   # one source chunk
    dst = torch.randint(0, n, (E,), generator=g, dtype=torch.int32)
    sh = G.build_shard(src.to(cuda), dst.to(cuda), n, 0, 1)
    lay = G.build_blocked(sh, 8192)
    assert lay.max_runs > 4096
    c = torch.rand(n, device=cuda)
    a1 = torch.zeros(sh.n_local, device=cuda)
    p1 = torch.zeros(sh.n_local, dtype=torch.int32, device=cuda)
    a2, p2 = torch.zeros_like(a1), torch.zeros_like(p1)
    G.pr_spmv(sh, c, a1, p1)
    G.pb_spmv(lay, c, a2, p2)
    torch.cuda.synchronize()
    assert torch.equal(p1, p2)
    assert torch.allclose(a1, a2, rtol=1e-6, atol=1e-7)


def test_pagerank_blocked_scale_matches_pull(cuda):
    """Whole PageRank runs (reference + standard semantics) on an R-MAT graph: blocked == pull."""
    from dalgo.apps.pagerank_app import rmat_shard
    from dalgo.models.pagerank import PageRank, PageRankConfig
    shard, _ = rmat_shard(16, 16, 0, 1, torch.device(cuda))
    for sem in ("reference", "standard"):
        rp = PageRank(PageRankConfig(semantics=sem, spmv="pull"), shard).fit()
        rb = PageRank(PageRankConfig(semantics=sem, spmv="blocked", chunk=1 << 12), shard).fit()
        assert torch.equal(rp.r >= 0, rb.r >= 0)
        assert torch.allclose(rp.r, rb.r, rtol=2e-5, atol=1e-12)


def test_pagerank_blocked_toy_and_standard(cuda):
    from dalgo.models.pagerank import PageRank, PageRankConfig
    from dalgo.ops import graph as G
    src = torch.tensor([0, 0, 1, 2], dtype=torch.int32, device=cuda)
    dst = torch.tensor([1, 2, 2, 0], dtype=torch.int32, device=cuda)
    r = PageRank(PageRankConfig(spmv="blocked"), G.build_shard(src, dst, 3, 0, 1)).fit().collect()
    assert r[0] == pytest.approx(0.38891305880091237, abs=1e-6)
    assert r[1] == pytest.approx(0.214416470596171, abs=1e-6)
    assert r[2] == pytest.approx(0.3966704706029163, abs=1e-6)


# ------------------------------------------------------------------ closure / ALS / MC
def test_transitive_closure_gpu(cuda):
    from dalgo.models.transitive_closure import DenseClosure, SparseClosure
    g = torch.Generator().manual_seed(2)
    n, e = 300, 420
    src = torch.randint(0, n, (e,), generator=g)
    dst = torch.randint(0, n, (e,), generator=g)
    ref = DenseClosure(src, dst, n).run().counts
    assert DenseClosure(src, dst, n, device=cuda).run().counts == ref
    assert SparseClosure(src, dst, n=n, device=cuda).run().counts == ref
    s4 = torch.tensor([0, 0, 1, 2])
    d4 = torch.tensor([1, 2, 2, 0])
    assert DenseClosure(s4, d4, 3, device=cuda).run().counts == [4, 8, 9, 9]
    # checkpoint after 3 rounds (bit-packed P^T slice / sparse path set), resume in a fresh
    # instance: the same trajectory as the uninterrupted run
    for cls in (DenseClosure, SparseClosure):
        kw = dict(n=n, device=cuda)
        a = cls(src, dst, **kw) if cls is SparseClosure else cls(src, dst, n, device=cuda)
        a.run(max_rounds=3)
        b = cls(src, dst, **kw) if cls is SparseClosure else cls(src, dst, n, device=cuda)
        b.load_state_dict(a.state_dict())
        assert b.run().counts == ref, cls.__name__


@pytest.mark.parametrize("n,nz", [(640, 384), (768, 512)])
def test_tc_step_kernel_exact(cuda, n, nz):
    """One K9 step (128 tiles at 640 x 384, 256 tiles at 768 x 512) == (T | (T A^T > 0))
    computed in f32 on the CPU."""
    from dalgo.ops import _ext
    g = torch.Generator().manual_seed(3)
    A = (torch.rand(n, n, generator=g) < 0.01).to(torch.uint8)
    T = (torch.rand(nz, n, generator=g) < 0.05).to(torch.uint8)
    ref = ((T != 0) | ((T.float() @ A.float().T) > 0.5)).to(torch.uint8)
    Tn = torch.zeros_like(T, device=cuda)
    cnt = torch.zeros(1, dtype=torch.int64, device=cuda)
    _ext.ops().tc_step(A.to(cuda), T.to(cuda), Tn, cnt)
    torch.cuda.synchronize()
    assert torch.equal(Tn.cpu(), ref)
    assert int(cnt.item()) == int(ref.sum())


def test_spd_inverse_gpu(cuda):
    from dalgo.models.als import spd_inverse
    for k in (10, 64, 128):
        A = torch.rand(200, k, dtype=torch.float64)
        G_ = (A.T @ A).float()
        inv = spd_inverse(G_.to(cuda), 5.0).cpu().double()
        ref = torch.linalg.inv(G_.double() + 5.0 * torch.eye(k, dtype=torch.float64))
        assert torch.allclose(inv, ref, rtol=1e-4, atol=1e-6)


# K5 als_solve: (R F) Ginv against f64, every launch variant (16x16x32 and 32x32x16 forms),
# k across 1..8 factor-column tiles, n not a multiple of 16 (tail K-step), rows not a multiple of
# the block, a strided (non-contiguous rows) R, a K-split count > 1
@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("m,n,k", [(100, 500, 10), (1000, 777, 64), (3000, 4096, 33),
                                   (600, 1000, 128), (513, 100, 96), (7, 5, 1), (20000, 3001, 64)])
def test_als_solve_gpu(cuda, monkeypatch, variant, m, n, k):
    from dalgo.models.als import rows_solve
    monkeypatch.setenv("DALGO_ALS_VARIANT", str(variant))
    g = torch.Generator().manual_seed(m * 7 + n + k)
    R = torch.rand(m, n, generator=g, dtype=torch.float64) * 16
    F = torch.rand(n, k, generator=g, dtype=torch.float64) - 0.3
    Gi = torch.rand(k, k, generator=g, dtype=torch.float64) - 0.5
    ref = (R @ F) @ Gi
    out = rows_solve(R.float().to(cuda), F.float().to(cuda), Gi.float().to(cuda)).cpu().double()
    # f32 rounding of the inputs + 2^-16 split residual, relative to sum |R||F||Gi|
    scale = (R.abs() @ F.abs()) @ Gi.abs()
    err = ((out - ref).abs() / scale).max().item()
    assert err < 2e-5, err
    if m > 64:   # strided rows (ld = n + 3 -> realigned copy inside rows_solve)
        Rs = torch.zeros(m, n + 3, dtype=torch.float32, device=cuda)[:, :n]
        Rs.copy_(R.float().to(cuda))
        out2 = rows_solve(Rs, F.float().to(cuda), Gi.float().to(cuda)).cpu().double()
        assert ((out2 - ref).abs() / scale).max().item() < 2e-5


@pytest.mark.parametrize("n,k", [(5, 1), (1000, 10), (70000, 64), (3000, 100), (2049, 128)])
def test_als_gram_gpu(cuda, n, k):
    """K5 split-n Gram F^T F against f64."""
    from dalgo.models.als import gram
    g = torch.Generator().manual_seed(n + k)
    F = torch.rand(n, k, generator=g, dtype=torch.float64) - 0.3
    ref = F.T @ F
    G = gram(F.float().to(cuda)).cpu().double()
    scale = F.abs().T @ F.abs()
    assert ((G - ref).abs() / scale.clamp_min(1e-30)).max().item() < 1e-5


@pytest.mark.parametrize("m,n,k", [(100, 500, 10), (513, 777, 64), (1000, 1001, 33), (7, 5, 1),
                                   (3000, 2000, 128), (4100, 96, 96)])
def test_als_residual_gpu(cuda, m, n, k):
    """K5 residual kernel: sum (R - U V^T)^2 with R close to U V^T (the cancelling regime),
    row / column tails, every K-step count, against f64."""
    from dalgo.ops import _ext
    g = torch.Generator().manual_seed(m + n + k)
    U = torch.rand(m, k, generator=g, dtype=torch.float64)
    V = torch.rand(n, k, generator=g, dtype=torch.float64)
    R = U @ V.T + 0.05 * (torch.rand(m, n, generator=g, dtype=torch.float64) - 0.5)
    Rf, Uf, Vf = R.float(), U.float(), V.float()
    ref = float(((Rf.double() - Uf.double() @ Vf.double().T) ** 2).sum())
    out = torch.zeros(1, dtype=torch.float64, device=cuda)
    ld = (n + 3) // 4 * 4
    Rd = torch.zeros(m, ld, dtype=torch.float32, device=cuda)[:, :n]
    Rd.copy_(Rf.to(cuda))
    _ext.ops().als_residual(Rd, Uf.to(cuda), Vf.to(cuda), out)
    assert abs(float(out.item()) - ref) / ref < 1e-3, (float(out.item()), ref)


def test_als_rmse_gpu_matches_f64(cuda):
    """ALS.rmse on the GPU (RV from the K5 GEMM, f64 dot and Grams) == the f64 residual
    norm of the same factors (m x n residual formed on the CPU)."""
    from dalgo.models.als import ALS, ALSConfig
    als = ALS(ALSConfig(m=3000, n=2000, k=16, seed=5), device=cuda)
    als.fit(2)
    R = (als.R_rows.cpu().double())
    res = R - als.U.cpu().double() @ als.V.cpu().double().T
    ref = math.sqrt(float((res ** 2).sum()) / (3000 * 2000))
    assert abs(als.rmse() - ref) / ref < 1e-3, (als.rmse(), ref)


def test_als_gpu(cuda):
    from dalgo.models.als import ALS, ALSConfig
    hc = ALS(ALSConfig(seed=3)).fit().rmse
    hg = ALS(ALSConfig(seed=3), device=cuda).fit().rmse
    assert hg[-1] < 0.05 and abs(hg[0] - hc[0]) < 1e-3


def test_monte_carlo_gpu(cuda):
    from dalgo.models.monte_carlo import MonteCarloConfig, estimate_pi
    pi_c, cnt_c = estimate_pi(MonteCarloConfig(n=2_000_000))
    pi_g, cnt_g = estimate_pi(MonteCarloConfig(n=2_000_000), device=cuda)
    assert abs(cnt_c - cnt_g) <= 4 and abs(pi_g - math.pi) < 0.01


# ------------------------------------------------------------------ LR family end-to-end
@pytest.mark.parametrize("algo", ["ssgd", "gd", "ma", "bmuf", "easgd"])
def test_lr_family_gpu_tracks_cpu(cuda, algo):
    from dalgo.data.datasets import synthetic_logistic
    from dalgo.models.localsgd import ParallelSGD, SGDConfig
    from dalgo.parallel import runtime
    from dalgo.parallel.sharding import make_layout
    rt = runtime.init(device="cuda")
    N, D = 40_000, 96
    cfg = SGDConfig(algo=algo, n_workers=4, n_iterations=15, eta=0.5, eval_every=0)
    lay = make_layout(N, 4, 1, 0, spark_compatible=False)
    dc = synthetic_logistic(N, D, dtype=torch.float32, device="cpu")
    dg = synthetic_logistic(N, D, dtype=torch.float32, device=cuda)
    assert torch.allclose(dg.X_train.cpu(), dc.X_train, atol=1e-6)
    mc = ParallelSGD(cfg, dc, lay, rt, model_dtype=torch.float64)
    mc.fit()
    mg = ParallelSGD(cfg, dg, lay, rt)
    mg.fit()
    a, b = mg.weights().cpu().double(), mc.weights()
    assert (a - b).norm() / b.norm() < 1e-4


@pytest.mark.parametrize("algo", ["ssgd", "gd", "ma", "bmuf", "easgd"])
@pytest.mark.parametrize("reuse", [True, False])
def test_lr_family_graph_replay_matches_eager(cuda, algo, reuse):
    """hipGraph replay (one captured step, device step counter) == eager launches:
    same minibatches (exact global sample count), same model up to f32 atomic order,
    including a checkpoint-style jump of t between replays."""
    if reuse is False and algo not in ("ma", "bmuf"):
        pytest.skip("reuse_minibatch only affects MA / BMUF")
    from dalgo.data.datasets import synthetic_logistic
    from dalgo.models.localsgd import ParallelSGD, SGDConfig
    from dalgo.parallel import runtime
    from dalgo.parallel.sharding import make_layout
    rt = runtime.init(device="cuda")
    N, D = 60_000, 200
    cfg = SGDConfig(algo=algo, n_workers=4, n_iterations=12, eta=0.5 if algo != "gd" else 1e-4,
                    eval_every=0, reuse_minibatch=reuse)
    lay = make_layout(N, 4, 1, 0, spark_compatible=False)
    d = synthetic_logistic(N, D, dtype=torch.bfloat16, device=cuda)
    runs = []
    for graph in (False, True):
        m = ParallelSGD(cfg, d, lay, rt)
        m.graph = graph
        m.count_acc = torch.zeros(1, dtype=torch.float64, device=cuda)
        m.fit(6)
        m.t += 3          # e.g. a resumed checkpoint: the device counter must follow
        m.fit(6)
        torch.cuda.synchronize()
        assert m._graph_ok() == graph
        if graph:
            assert len(m._graphs) == 1
        runs.append((m.weights().clone(), float(m.count_acc.item()), m.t))
    (we, ce, te), (wg, cg, tg) = runs
    assert te == tg == 15
    if algo in ("ssgd", "gd"):
        assert ce == cg
    rel = ((wg - we).norm() / we.norm()).item()
    assert rel < 1e-4, rel


@pytest.mark.parametrize("n,e,seed", [(3000, 2600, 1), (20000, 18000, 2), (2500, 3750, 3)])
def test_sparse_closure_gpu_exact(cuda, n, e, seed):
    """K9 sparse (hash-set frontier join): per-round path counts == the CPU torch engine,
    the final path SET equal too; the third graph is supercritical (large closure, the
    hash set grows several times)."""
    from dalgo.models.transitive_closure import SparseClosure
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, n, (e,), generator=g)
    dst = torch.randint(0, n, (e,), generator=g)
    cpu = SparseClosure(src, dst, n=n)
    gpu = SparseClosure(src, dst, n=n, device=cuda)
    assert gpu.run().counts == cpu.run().counts
    assert torch.equal(gpu.paths().cpu(), cpu.paths())


def test_sparse_closure_expand_skewed_degrees(cuda):
    """One expansion over a frontier whose candidate prefix has long runs of zero-degree
    paths (blocks spanning > 2048 frontier entries: global binary search) and hubs with
    tens of thousands of in-edges (one path spans many blocks) == torch join."""
    from dalgo.models.transitive_closure import SparseClosure
    g = torch.Generator().manual_seed(7)
    n = 100_000
    hubs = torch.tensor([5, 77, 4242])
    src = torch.cat([torch.randint(0, n, (60_000,), generator=g),
                     torch.randint(0, n, (3000,), generator=g)])
    dst = torch.cat([hubs[torch.randint(0, 3, (60_000,), generator=g)],
                     torch.randint(0, n, (3000,), generator=g)])
    # initial paths: the edges; frontier sources mostly have in-degree 0
    cpu = SparseClosure(src, dst, n=n)
    gpu = SparseClosure(src, dst, n=n, device=cuda)
    for _ in range(3):
        assert gpu.step() == cpu.step()
        assert torch.equal(gpu.frontier().cpu(), cpu.frontier())
    assert int(gpu.err.item()) == 0


def test_sparse_closure_gpu_resume(cuda):
    from dalgo.models.transitive_closure import SparseClosure
    g = torch.Generator().manual_seed(11)
    n, e = 5000, 4700
    src = torch.randint(0, n, (e,), generator=g)
    dst = torch.randint(0, n, (e,), generator=g)
    ref = SparseClosure(src, dst, n=n, device=cuda).run().counts
    a = SparseClosure(src, dst, n=n, device=cuda)
    a.run(max_rounds=4)
    b = SparseClosure(src, dst, n=n, device=cuda)
    b.load_state_dict(a.state_dict())
    assert b.run().counts == ref


@pytest.mark.parametrize("d,dtype", [(64, torch.bfloat16), (128, torch.bfloat16), (30, torch.float32)])
def test_kmeans_incremental_accumulate_exact(cuda, d, dtype):
    """Incremental K3 (moved rows only, f64 local sums): after every iteration the counts
    equal a full K3 pass over the same assignment exactly, and the sums equal the first
    (full, f32) pass plus the exact f64 change of the per-cluster sums since then: the
    moves add no error of their own."""
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.ops import kmeans as K
    n, k = 150_000, 96
    X = blobs(n, d, k, device=cuda, dtype=dtype, seed=5)
    km = KMeans(KMeansConfig(k=k, n_iterations=6, seed=2, bound_filter=False), X, 0, n)
    assert km.incremental and not km.bounds

    def exact(a):
        S = torch.zeros(k, km.DP, dtype=torch.float64, device=cuda)
        S[:, :d].index_add_(0, a.long(), km.X.double())
        return S

    c_ref = torch.zeros_like(km.cnt)
    S_ref = torch.zeros_like(km.S)
    for it in range(6):
        km.step()
        if it == 0:
            S0, E0 = km.S.double().clone(), exact(km.assign)
        c_ref.zero_()
        S_ref.zero_()
        K.accumulate(km.X, km.assign, k, km.DP, S_ref, c_ref)
        assert torch.equal(km.cnt, c_ref), it
        expect = S0 + (exact(km.assign) - E0)
        assert torch.allclose(km.S.double(), expect, rtol=1e-6, atol=1e-2), it
    assert len(km.changed_history) == 5 and km.changed_history[0] > 0


@pytest.mark.parametrize("d,dtype,k,m", [(128, torch.bfloat16, 1024, 300_000),
                                         (64, torch.bfloat16, 96, 40_000),
                                         (30, torch.float32, 2048, 20_000),
                                         (128, torch.bfloat16, 1024, 3),
                                         (64, torch.bfloat16, 512, 0)])
def test_kmeans_move_sorted_exact(cuda, d, dtype, k, m):
    """Sort-based incremental K3 with the moved-row count on the DEVICE (workspace sized for
    every row): sums / counts / |x|^2 sums Q == the f64 signed moves computed by torch."""
    n = 500_000
    g = torch.Generator().manual_seed(3)
    X = K.prepare_points((torch.randn(n, d, generator=g) * 3).to(dtype).to(cuda))
    DP = K.kmeans_dp(d)
    a_old = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(cuda)
    a_new = a_old.clone()
    rows = torch.randperm(n, generator=g)[:m].to(cuda)
    a_new[rows] = torch.randint(0, k, (m,), generator=g, dtype=torch.int32).to(cuda)
    changed = torch.zeros(n, dtype=torch.int32, device=cuda)
    changed[:m] = torch.sort(rows.to(torch.int32)).values
    m_dev = torch.tensor([m], dtype=torch.int64, device=cuda)
    xh = (torch.rand(n, generator=g) * 10).to(cuda)
    ws = K.MoveWorkspace(cuda, n, k)
    S = torch.zeros(k, DP, dtype=torch.float64, device=cuda)
    c = torch.zeros(k, dtype=torch.int64, device=cuda)
    Q = torch.zeros(k, dtype=torch.float64, device=cuda)
    K.move_rows(X, DP, changed, m_dev, a_new, a_old, S, c, ws, xh, Q)
    r = rows.long()
    xr = X[r].double()
    Se = torch.zeros(k, DP, dtype=torch.float64, device=cuda)
    Se[:, :d].index_add_(0, a_new[r].long(), xr)
    Se[:, :d].index_add_(0, a_old[r].long(), -xr)
    ce = torch.bincount(a_new[r].long(), minlength=k) - torch.bincount(a_old[r].long(), minlength=k)
    Qe = torch.zeros(k, dtype=torch.float64, device=cuda)
    Qe.index_add_(0, a_new[r].long(), 2.0 * xh[r].double())
    Qe.index_add_(0, a_old[r].long(), -2.0 * xh[r].double())
    assert torch.equal(c, ce)
    assert torch.allclose(S, Se, rtol=1e-12, atol=1e-9), (S - Se).abs().max()
    assert torch.allclose(Q, Qe, rtol=1e-12, atol=1e-6), (Q - Qe).abs().max()


def test_kmeans_assign_rows_indirect(cuda):
    """K2 with row indirection (only the listed rows) == the full K2 on those rows, and
    leaves every other row's assignment untouched."""
    torch.manual_seed(5)
    n, d, k = 50_000, 128, 1000
    X = K.prepare_points((torch.randn(n, d) * 3).to(torch.bfloat16).to(cuda))
    cen = K.make_centers(torch.randn(k, d) * 3, torch.bfloat16, cuda)
    full = K.assign(X, cen)
    rows = torch.randperm(n, device=cuda)[: n // 3].to(torch.int32)
    a = torch.full((n,), -7, dtype=torch.int32, device=cuda)
    mind = torch.zeros(n, device=cuda)
    K.assign_rows(X, cen, rows, rows.numel(), a, mind)
    sel = torch.zeros(n, dtype=torch.bool, device=cuda)
    sel[rows.long()] = True
    assert torch.equal(a[sel], full[sel])
    assert bool((a[~sel] == -7).all()) and bool((mind[sel] > 0).all())


def test_kmeans_filter_matches_torch(cuda):
    """Bound filter (maxd reduced in-kernel from delta, bounds rounded outward) == torch;
    the active count stays on the device; with acl, the kept rows' clusters in list order."""
    torch.manual_seed(6)
    n, k = 100_003, 50
    assign = torch.randint(0, k, (n,), dtype=torch.int32, device=cuda)
    ul = torch.stack([torch.rand(n, device=cuda) * 10, torch.rand(n, device=cuda) * 20], 1)
    u, l = ul[:, 0], ul[:, 1]                   # views: the kernel updates ul in place
    delta = torch.rand(k, device=cuda)
    s = torch.rand(k, device=cuda) * 12
    maxd = delta.max()
    u0, l0 = u.clone(), l.clone()
    a_prev = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    idx = torch.empty(n, dtype=torch.int32, device=cuda)
    cnt = torch.zeros(1, dtype=torch.int64, device=cuda)
    acl = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    K.filter_rows(assign, ul, delta, s, a_prev, idx, cnt, acl)
    m = int(cnt.item())
    assert torch.equal(acl[:m], assign[idx[:m].long()])
    ub = u0 + delta[assign.long()]
    lb = l0 - maxd
    act = ~(ub < torch.maximum(s[assign.long()], lb))
    # outward rounding can only add active rows at exact float ties: none in random data
    assert m == int(act.sum())
    assert torch.equal(torch.sort(idx[:m]).values.long(), torch.nonzero(act)[:, 0])
    assert bool((u[~act] >= ub[~act]).all()) and torch.allclose(u[~act], ub[~act])
    assert bool((l[~act] <= lb[~act]).all()) and torch.allclose(l[~act], lb[~act])
    assert torch.equal(u[act], u0[act]) and torch.equal(l[act], l0[act])
    assert torch.equal(a_prev[act], assign[act])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("k,d", [(1, 8), (7, 30), (1024, 128)])
def test_kmeans_centre_bounds_kernel(cuda, dtype, k, d):
    """delta / s of the bound filter (one launch) == f64 torch, rounded outward."""
    torch.manual_seed(k + d)
    DP = K.kmeans_dp(d)
    a = torch.zeros(K.make_centers(torch.zeros(k, d), dtype, "cpu").Cq.shape, dtype=dtype)
    a[:k, :d] = (torch.randn(k, d) * 3).to(dtype)
    b = a.clone()
    b[:k, :d] = (a[:k, :d].float() + torch.randn(k, d) * 0.1).to(dtype)
    dg, sg = K.centre_bounds(a.to(cuda), b[:k].contiguous().to(cuda), k, d)
    dc, sc = K.centre_bounds(a, b[:k].contiguous(), k, d)
    ad, bd = a[:k, :d].double(), b[:k, :d].double()
    dex = (ad - bd).norm(dim=1)
    assert bool((dg.cpu().double() >= dex).all())
    assert torch.allclose(dg.cpu(), dc, rtol=1e-5, atol=1e-6)
    if k == 1:
        assert bool(torch.isinf(sg).all())
    else:
        dd = torch.cdist(ad, ad)
        dd.fill_diagonal_(float("inf"))
        assert bool((sg.cpu().double() <= 0.5 * dd.min(dim=1).values).all())
        assert torch.allclose(sg.cpu(), sc, rtol=1e-5)


@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("prev", ["a_prev", "acl", "assign"])
def test_kmeans_assign_rows_fused_post(cuda, prev, d):
    """Filtered-iteration K2 (row count on the device, fused bound update; d = 128: the
    dense 16x16x32 top-2 form): only idx[:*m_dev] is re-assigned, equal to the full pass
    on those rows; u / l bracket the exact distances (rounded outward, tol on the device);
    the changed rows (vs the previous cluster: a_prev[row], acl[p] in list order, or
    assign[row] itself) are collected exactly, with their new / previous clusters. Also
    the full pass's optional 0.5|x|^2 / max outputs and the bounds-init kernel. d = 64:
    the pipelined 32x32x16 form."""
    torch.manual_seed(9)
    n, k = 60_001, 1000
    X = K.prepare_points((torch.randn(n, d) * 3).to(torch.bfloat16).to(cuda))
    cen = K.make_centers(torch.randn(k, d) * 3, torch.bfloat16, cuda)
    full = K.assign(X, cen)
    # full pass: top-2 distances, xh, xmax, then the bounds init
    a0 = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.zeros(n, device=cuda)
    mind2 = torch.zeros(n, device=cuda)
    xh = torch.zeros(n, device=cuda)
    xmax = torch.zeros(1, dtype=torch.int32, device=cuda)
    K.assign_rows(X, cen, None, n, a0, mind, mind2, xh=xh, xmax=xmax)
    ref = 0.5 * X[:, :d].float().pow(2).sum(1)
    assert torch.allclose(xh, ref, rtol=1e-5)
    assert float(xmax.view(torch.float32).item()) == pytest.approx(float(ref.max()), rel=1e-5)
    ul0 = torch.empty((n, 2), device=cuda)
    u0, l0 = ul0[:, 0], ul0[:, 1]
    tol = torch.zeros(1, device=cuda)
    K.bounds_init(mind, mind2, xmax, n, ul0, tol)
    t = float(tol.item())
    assert t == pytest.approx(2 * (float(ref.max()) * 1.0001 + 1e-6) * 2 ** -14, rel=1e-5)
    assert bool((u0 >= torch.sqrt(mind + t)).all()) and bool((l0 <= torch.sqrt((mind2 - t).clamp_min(0))).all())
    # filtered form over a random subset, a_prev = a perturbed copy of the truth
    rows = torch.randperm(n, device=cuda).to(torch.int32)
    m = 23_457
    a_prev = full.clone()
    flip = torch.zeros(n, dtype=torch.bool, device=cuda)
    flip[rows[: m // 3].long()] = True          # a third of the active rows "moved"
    a_prev[flip] = (a_prev[flip] + 1) % k
    sel = torch.zeros(n, dtype=torch.bool, device=cuda)
    sel[rows[:m].long()] = True
    # assign holds the previous clusters of the active rows: only the changed ones are written
    a = torch.where(sel, a_prev, torch.full_like(a_prev, -7))
    ul = torch.full((n, 2), -1.0, device=cuda)
    u, l = ul[:, 0], ul[:, 1]
    changed = torch.empty(n, dtype=torch.int32, device=cuda)
    nch = torch.zeros(1, dtype=torch.int64, device=cuda)
    cnew = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    cold = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    post = dict(m_dev=torch.tensor([m], dtype=torch.int64, device=cuda), tol=tol, ul=ul,
                changed=changed, n_changed=nch, chg_new=cnew, chg_old=cold)
    if prev == "a_prev":
        post["a_prev"] = a_prev
    elif prev == "acl":
        acl = torch.full((n,), -3, dtype=torch.int32, device=cuda)
        acl[:m] = a_prev[rows[:m].long()]
        post["acl"] = acl
    K.assign_rows(X, cen, rows, n, a, post=post)
    assert torch.equal(a[sel], full[sel]) and bool((a[~sel] == -7).all())
    assert bool((u[~sel] == -1).all()) and bool((l[~sel] == -1).all())
    dist = torch.cdist(X[:, :d].double(), cen.Cq[:k, :d].double())
    two = torch.topk(dist, 2, dim=1, largest=False).values
    slack = 2 * t
    assert bool((u[sel].double() >= two[sel, 0] - 1e-3).all())
    assert bool((u[sel].double() <= torch.sqrt(two[sel, 0] ** 2 + slack) + 1e-3).all())
    assert bool((l[sel].double() <= two[sel, 1] + 1e-3).all())
    c = int(nch.item())
    exp = torch.nonzero(sel & (full != a_prev))[:, 0]
    assert c == exp.numel()
    assert torch.equal(torch.sort(changed[:c]).values.long(), exp)
    rows_c = changed[:c].long()
    assert torch.equal(cnew[:c], full[rows_c]) and torch.equal(cold[:c], a_prev[rows_c])


def test_kmeans_assign_top2_second_best(cuda):
    """Top-2 K2: the second-best distance is a lower bound of (and within rounding of) the
    true second-smallest distance to the rounded centres; the best is unchanged."""
    torch.manual_seed(8)
    n, d, k = 40_000, 128, 1000
    X = K.prepare_points((torch.randn(n, d) * 3).to(torch.bfloat16).to(cuda))
    cen = K.make_centers(torch.randn(k, d) * 3, torch.bfloat16, cuda)
    full = K.assign(X, cen)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.empty(n, device=cuda)
    mind2 = torch.empty(n, device=cuda)
    K.assign_rows(X, cen, None, n, a, mind, mind2)
    assert (a == full).float().mean().item() > 0.999
    dist = torch.cdist(X[:, :d].double(), cen.Cq[:k, :d].double()) ** 2
    two = torch.topk(dist, 2, dim=1, largest=False).values
    tol = 1e-3 * (1 + float(dist.max()))
    assert bool((mind2.double() <= two[:, 1] + tol).all())
    assert float((two[:, 1] - mind2.double()).abs().max()) < tol
    assert bool((mind2 >= mind - tol).all())


def test_kmeans_bound_filter_exact(cuda):
    """Bound-filtered Lloyd (default for bf16 on the GPU): every step equals brute force
    from the same state (near-ties within the rounding slack aside) with exact counts and
    sums; SSE trajectory (Q identity) vs plain Lloyd; the filter skips most points once
    the centres settle."""
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    n, d, k = 300_000, 128, 1000
    X = blobs(n, d, k, device=cuda, dtype=torch.bfloat16, seed=11)
    a = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, candidates=False), X, 0, n)
    assert a.bounds
    a.fit()
    b = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, bound_filter=False), X, 0, n)
    assert not b.bounds
    b.fit()
    assert np.allclose(a.history.sse, b.history.sse, rtol=2e-4), (a.history.sse, b.history.sse)
    assert a.active_history[0] == n and min(a.active_history[1:]) < 0.3 * n
    # the oracle: every filtered step, from its own centres and bounds, against the
    # brute-force full pass over the same centres (plus exact counts and sums)
    c = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, candidates=False), X, 0, n)
    for _ in range(7):
        _kmeans_step_oracle(c)


def _kmeans_step_oracle(km):
    """One step of ``km`` checked against brute force from the same state: the K2
    assignment over the centres the step used differs from the full-pass K2 only at
    near-ties (distance gap within the kernels' rounding slack), the counts equal a K3
    pass over the step's assignment exactly and the maintained sums equal the f64 sums."""
    from dalgo.ops import kmeans as K
    k, d = km.cfg.k, km.d
    cq = km.cen.Cq.clone()
    km.step()
    used = K.make_centers(cq[:k, :d].float(), km.X.dtype, km.dev, kpad=cq.shape[0])
    a_full = K.assign(km.X, used)
    diff = (a_full != km.assign).nonzero().flatten()
    assert diff.numel() <= max(5, km.X.shape[0] // 2000), diff.numel()
    if diff.numel():
        Xd = km.X[diff, :d].double()
        Cd = cq[:k, :d].double()
        gap = ((Xd - Cd[km.assign[diff].long()]).pow(2).sum(1) -
               (Xd - Cd[a_full[diff].long()]).pow(2).sum(1)).abs()
        xmax = float((km.X[:, :d].float().pow(2).sum(1).max() * 0.5).item())
        slack = 2.0 * (xmax * 1.0001 + 1e-6) * 2.0 ** -14 * 2.0
        assert float(gap.max()) <= slack, (float(gap.max()), slack)
    S_ref = torch.zeros_like(km.S)
    c_ref = torch.zeros_like(km.cnt)
    K.accumulate(km.X, km.assign, k, km.DP, S_ref, c_ref)
    S_m = km._S64 if km.incremental else km.S.double()
    c_m = km._cnt64 if km.incremental else km.cnt
    assert torch.equal(c_ref, c_m)
    S_ex = torch.zeros(k, km.DP, dtype=torch.float64, device=km.dev)
    S_ex[:, :d].index_add_(0, km.assign.long(), km.X[:, :d].double())
    rel = float(((S_m.double() - S_ex).abs().max() / (1.0 + S_ex.abs().max())).item())
    assert rel < 1e-5, rel


@pytest.mark.parametrize("k,d", [(1, 8), (37, 30), (1024, 128)])
def test_kmeans_centre_nbrs_kernel(cuda, k, d):
    """Neighbour lists of the candidate-pruned K2: nd ascending lower bounds of the centre
    distances, nb = the same order with each aligned 32-group re-ordered by id, hnb
    gathered through nb; delta / s equal the plain centre-bounds kernel's."""
    torch.manual_seed(k + d)
    cen = K.make_centers(torch.randn(k, d) * 3, torch.bfloat16, cuda)
    kpad, DP = cen.Cq.shape
    prev = cen.Cq[:k].clone()
    prev[:, :d] = (prev[:, :d].float() + 0.1 * torch.randn(k, d, device=cuda)).to(torch.bfloat16)
    ws = K.CandWorkspace(cuda, 1000, k, kpad, DP, drift=True)
    delta = torch.empty(k, device=cuda)
    s = torch.empty(k, device=cuda)
    K.centre_nbrs(cen, prev, delta, s, ws)
    # drift-aware lists: each entry's own distance (rounded down) and its centre's shift
    nbl = ws.nb.view(k, kpad).long()
    Dl = torch.cdist(cen.Cq[:k, :d].double(), cen.Cq[:k, :d].double())
    ndb = ws.ndb.view(k, kpad)
    real = nbl < k
    got_d = Dl.gather(1, nbl.clamp(max=k - 1))
    assert bool((ndb[real].double() <= got_d[real] + 1e-9).all())
    assert torch.allclose(ndb[real].double(), got_d[real], rtol=1e-5, atol=1e-5)
    assert bool(torch.isinf(ndb[~real]).all())
    assert torch.equal(ws.dnb.view(k, kpad)[real], delta[nbl[real]])
    d0, s0 = K.centre_bounds(cen.Cq, prev, k, d)
    assert torch.equal(delta, d0) and torch.equal(s, s0)
    C = cen.Cq[:k, :d].double()
    D = torch.cdist(C, C)
    nd = ws.nd.view(k, kpad)
    nb = ws.nb.view(k, kpad).long()
    assert bool((nd[:, 1:] >= nd[:, :-1]).all())
    assert bool(torch.isinf(nd[:, k:]).all())
    sd = torch.sort(D, dim=1).values
    assert bool((nd[:, :k].double() <= sd + 1e-9).all())
    assert torch.allclose(nd[:, :k].double(), sd, rtol=1e-5, atol=1e-5)
    for g in range(0, kpad, 32):
        grp = nb[:, g:g + 32]
        assert bool((grp[:, 1:] > grp[:, :-1]).all())            # ids ascending per group
    # each group holds the centres of those distance ranks
    got = torch.where(nb < k, D.gather(1, nb.clamp(max=k - 1)),
                      torch.full(nb.shape, float("inf"), dtype=torch.float64, device=cuda))
    for g in range(0, kpad, 32):
        hi = torch.sort(got[:, g:g + 32], dim=1).values
        ref = torch.cat([sd, torch.full((k, kpad - k), float("inf"), device=cuda, dtype=torch.float64)], 1)[:, g:g + 32]
        assert torch.allclose(hi, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(ws.hnb.view(k, kpad), cen.hn[nb])


def test_kmeans_sort_active(cuda):
    """Active rows counting-sorted by cluster with a device count, cluster runs and the
    tile table (tiles never straddle clusters)."""
    torch.manual_seed(4)
    n, k, m = 300_001, 97, 123_457
    ws = K.CandWorkspace(cuda, n, k, 128, 64)
    idx = torch.randperm(n, device=cuda).to(torch.int32)
    ws.acl.copy_(torch.randint(0, k, (n,), device=cuda, dtype=torch.int32))
    cnt = torch.tensor([m], dtype=torch.int64, device=cuda)
    K.sort_active(idx, cnt, ws)
    acl, rows = ws.acl[:m].long(), ws.rows[:m].long()
    cl_of_row = torch.full((n,), -1, dtype=torch.long, device=cuda)
    cl_of_row[idx[:m].long()] = acl
    assert torch.equal(torch.sort(rows).values, torch.sort(idx[:m].long()).values)
    cs = ws.cstart
    assert torch.equal(cs, torch.cat([torch.zeros(1, dtype=torch.long, device=cuda),
                                      torch.cumsum(torch.bincount(acl, minlength=ws.nkeys), 0)]))
    rc = cl_of_row[rows]
    assert bool((rc[1:] >= rc[:-1]).all())
    T = int(ws.n_tiles.item())
    ref = sum((int(cs[c + 1] - cs[c]) + K.CAND_TILE - 1) // K.CAND_TILE for c in range(ws.nkeys))
    assert T == ref
    tr = ws.tiles.view(-1, 4)[:T].long()
    tc, tl, th = tr[:, 0], tr[:, 1], tr[:, 2]
    assert bool((tl >= cs[tc]).all()) and bool((tl < cs[tc + 1]).all())
    assert bool(((tl - cs[tc]) % K.CAND_TILE == 0).all())
    assert torch.equal(th, torch.minimum(cs[tc + 1], tl + K.CAND_TILE))
    assert int((th - tl).sum()) == m


@pytest.mark.parametrize("d,tile16", [(64, False), (128, False), (128, True)])
def test_kmeans_assign_rows_candidates(cuda, d, tile16):
    """Candidate-pruned filtered K2 (tiles of one cluster stream only the centres within
    2 max(u) + slack of their centre): same assignment as the full pass on the active
    rows (mismatches only at kernel-rounding near-ties), the pruned centres bound l from
    below, the changed rows are collected exactly. tile16: the 16x16x32 form (384-row
    tiles, kmeans_assign16_kernel CND)."""
    torch.manual_seed(12)
    from dalgo.data.synthetic import blobs
    n, k = 120_000, 512
    X = K.prepare_points(blobs(n, d, k, device=cuda, dtype=torch.bfloat16, seed=4))
    g = torch.Generator(device="cpu").manual_seed(2)
    C0 = X[torch.randperm(n, generator=g)[:k].to(cuda), :d].float()
    cen = K.make_centers(C0 + 0.5 * torch.randn_like(C0), torch.bfloat16, cuda)
    full = K.assign(X, cen)
    a0 = torch.empty(n, dtype=torch.int32, device=cuda)
    mind = torch.zeros(n, device=cuda)
    mind2 = torch.zeros(n, device=cuda)
    xmax = torch.zeros(1, dtype=torch.int32, device=cuda)
    K.assign_rows(X, cen, None, n, a0, mind, mind2, xh=torch.zeros(n, device=cuda), xmax=xmax)
    tol = torch.zeros(1, device=cuda)
    K.bounds_init(mind, mind2, xmax, n, torch.empty((n, 2), device=cuda), tol)
    kpad, DP = cen.Cq.shape
    ws = K.CandWorkspace(cuda, n, k, kpad, DP, tile=K.CAND16_TILE if tile16 else K.CAND_TILE)
    K.centre_nbrs(cen, cen.Cq[:k].clone(), torch.empty(k, device=cuda), torch.empty(k, device=cuda), ws)
    # active rows: a random subset; a_prev = the truth with a third of them perturbed, u =
    # a valid upper bound of the distance to c_{a_prev}
    m = 50_001
    rows = torch.randperm(n, device=cuda)[:m].to(torch.int32)
    a_prev = full.clone()
    flip = torch.zeros(n, dtype=torch.bool, device=cuda)
    flip[rows[: m // 3].long()] = True
    a_prev[flip] = (a_prev[flip] + 1) % k
    dprev = (X[:, :d].float() - cen.Cq[a_prev.long(), :d].float()).norm(dim=1)
    ul = torch.stack([dprev * 1.001 + 1e-3, torch.full((n,), -1.0, device=cuda)], 1)
    u, l = ul[:, 0], ul[:, 1]
    ws.acl[:m].copy_(a_prev[rows.long()])
    cnt = torch.tensor([m], dtype=torch.int64, device=cuda)
    K.sort_active(rows, cnt, ws)
    sel = torch.zeros(n, dtype=torch.bool, device=cuda)
    sel[rows.long()] = True
    # assign holds the previous clusters of the active rows: only the changed ones are written
    a = torch.where(sel, a_prev, torch.full_like(a_prev, -7))
    changed = torch.empty(n, dtype=torch.int32, device=cuda)
    cnew = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    cold = torch.full((n,), -1, dtype=torch.int32, device=cuda)
    nch = torch.zeros(1, dtype=torch.int64, device=cuda)
    K.assign_rows(X, cen, ws.rows, n, a, post=dict(
        m_dev=cnt, a_prev=None, tol=tol, ul=ul, changed=changed, n_changed=nch,
        chg_new=cnew, chg_old=cold), cand=ws)
    assert bool((a[~sel] == -7).all())
    dist = torch.cdist(X[:, :d].double(), cen.Cq[:k, :d].double())
    bad = sel & (a != full)
    if bool(bad.any()):
        db = dist[bad].gather(1, a[bad].long()[:, None])[:, 0]
        df = dist[bad].gather(1, full[bad].long()[:, None])[:, 0]
        assert float(((db - df).abs() / df).max()) < 1e-4
    assert int(bad.sum()) <= (10 if tile16 else 5)   # near-ties (the gap check above)
    two = torch.topk(dist, 2, dim=1, largest=False).values
    t = float(tol.item())
    assert bool((u[sel].double() >= two[sel, 0] - 1e-3).all())
    assert bool((u[sel].double() <= torch.sqrt(two[sel, 0] ** 2 + 2 * t) + 1e-3).all())
    assert bool((l[sel].double() <= two[sel, 1] + 1e-3).all())
    assert bool((l[sel] >= 0).all())
    c = int(nch.item())
    exp = torch.nonzero(sel & (a != a_prev))[:, 0]
    assert c == exp.numel()
    assert torch.equal(torch.sort(changed[:c]).values.long(), exp)
    # the moved rows' clusters travel next to them (no a_prev array was given)
    rows_c = changed[:c].long()
    assert torch.equal(cnew[:c], a[rows_c]) and torch.equal(cold[:c], a_prev[rows_c])


def test_kmeans_candidates_match_plain(cuda):
    """Filtered Lloyd with candidate-pruned tiles: every step equals brute force from
    the same state (near-ties within the rounding slack aside); the SSE trajectories of
    the pruned, bound-only and plain runs agree."""
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    n, d, k = 300_000, 128, 1000
    X = blobs(n, d, k, device=cuda, dtype=torch.bfloat16, seed=11)
    runs = {}
    for name, kw in [("cand", {}), ("bounds", dict(candidates=False)),
                     ("plain", dict(bound_filter=False)), ("dense", dict(dense="always")),
                     ("cand_nodrift", dict(drift=False)), ("cand_never", dict(dense="never"))]:
        km = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, **kw), X, 0, n)
        km.fit()
        runs[name] = km
    assert runs["cand"]._cand is not None and runs["bounds"]._cand is None
    assert runs["cand"]._cand.ndb is not None and runs["cand_nodrift"]._cand.ndb is None
    for other in ("bounds", "plain", "dense", "cand_nodrift", "cand_never"):
        assert np.allclose(runs["cand"].history.sse, runs[other].history.sse, rtol=2e-4)
    ha, hb = runs["cand"].active_history, runs["bounds"].active_history
    assert ha[0] == n and len(ha) == len(hb)
    # the oracle: every candidate-pruned step (the dense one right after the full pass
    # included) against brute force from the same state; then the dense form on every step
    for kw in ({}, dict(dense="always"), dict(dense="never"), dict(dense="never", drift=False)):
        c = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, **kw), X, 0, n)
        assert c._cand is not None
        for _ in range(7):
            _kmeans_step_oracle(c)


@pytest.mark.parametrize("c16", ["1", "0"])
def test_kmeans_cand16_matches_plain(cuda, monkeypatch, c16):
    """Both candidate-pruned K2 forms (DALGO_KM_CAND16=1: the 16x16x32 tiling, the default;
    0: the 32x32x16 pipelined form): every filtered step equals brute force from the same
    state, and the SSE trajectory equals the plain Lloyd run's."""
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    n, d, k = 300_000, 128, 1000
    X = blobs(n, d, k, device=cuda, dtype=torch.bfloat16, seed=11)
    plain = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, bound_filter=False), X, 0, n)
    plain.fit()
    monkeypatch.setenv("DALGO_KM_CAND16", c16)
    for kw in ({}, dict(dense="never"), dict(dense="never", drift=False)):
        km = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, **kw), X, 0, n)
        assert km._cand is not None
        assert km._cand.tile == (K.CAND16_TILE if c16 == "1" else K.CAND_TILE)
        assert (km._cand.ndb is None) == (kw.get("drift") is False)
        km.fit()
        assert np.allclose(km.history.sse, plain.history.sse, rtol=2e-4)
        c = KMeans(KMeansConfig(k=k, n_iterations=7, seed=5, **kw), X, 0, n)
        for _ in range(7):
            _kmeans_step_oracle(c)


def test_kmeans_dense_choice_on_device(cuda):
    """Filtered iterations pick the dense top-2 K2 or the pruned one on the device: right
    after the full pass always dense, later dense iff >= DENSE_FRACTION of the rows are
    active (dense_history = rows the dense K2 took, 0 otherwise); "never" / "always"
    force one form; every run passes the one-step oracle."""
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import DENSE_FRACTION, KMeans, KMeansConfig
    n, d, k = 200_000, 128, 512
    X = blobs(n, d, k, device=cuda, dtype=torch.bfloat16, seed=13, noise=2.0)
    for mode in ("auto", "never", "always"):
        # (the plain candidate lists: the device choice at DENSE_FRACTION; the drift-aware
        # lists use the same mechanism at DENSE_FRACTION_DRIFT)
        km = KMeans(KMeansConfig(k=k, n_iterations=6, seed=3, dense=mode, drift=False), X, 0, n)
        assert km._cand is not None
        for _ in range(6):
            _kmeans_step_oracle(km)
        act, dense = km.active_history, km.dense_history
        assert dense[0] == 0                                   # the full pass
        for i in range(1, len(act)):
            if mode == "never":
                want = 0
            elif mode == "always" or i == 1:
                want = act[i]
            else:
                want = act[i] if act[i] >= DENSE_FRACTION * n else 0
            assert dense[i] == want, (mode, i, act, dense)
        if mode == "auto":   # this data exercises both device choices (probe: r5_34)
            assert any(dense[i] > 0 for i in range(2, len(act))), (act, dense)
            assert any(dense[i] == 0 for i in range(2, len(act))), (act, dense)


@pytest.mark.parametrize("d,tile16", [(64, False), (128, False), (128, True)])
def test_kmeans_assign_rows_drift_candidates(cuda, d, tile16):
    """Drift-aware candidate lists: with valid lower bounds l (below the true second-best
    distance) and small centre shifts most of every list is dropped past the first chunk;
    the assignment still equals the full pass on the active rows (near-ties aside), u / l
    stay valid bounds and the changed rows are collected exactly."""
    torch.manual_seed(13)
    from dalgo.data.synthetic import blobs
    n, k = 120_000, 1000
    X = K.prepare_points(blobs(n, d, k, device=cuda, dtype=torch.bfloat16, seed=6))
    g = torch.Generator(device="cpu").manual_seed(3)
    C0 = X[torch.randperm(n, generator=g)[:k].to(cuda), :d].float()
    prevc = K.make_centers(C0, torch.bfloat16, cuda)
    cen = K.make_centers(C0 + 0.05 * torch.randn_like(C0), torch.bfloat16, cuda)
    full = K.assign(X, cen)
    kpad, DP = cen.Cq.shape
    xmax = torch.zeros(1, dtype=torch.int32, device=cuda)
    mind = torch.zeros(n, device=cuda)
    K.assign_rows(X, cen, None, n, torch.empty(n, dtype=torch.int32, device=cuda), mind,
                  torch.zeros(n, device=cuda), xh=torch.zeros(n, device=cuda), xmax=xmax)
    tol = torch.zeros(1, device=cuda)
    K.bounds_init(mind, mind, xmax, n, torch.empty((n, 2), device=cuda), tol)
    ws = K.CandWorkspace(cuda, n, k, kpad, DP, drift=True, tile=K.CAND16_TILE if tile16 else K.CAND_TILE)
    delta = torch.empty(k, device=cuda)
    K.centre_nbrs(cen, prevc.Cq[:k].clone(), delta, torch.empty(k, device=cuda), ws)
    # previous assignment / bounds vs the PREVIOUS centres: a_prev = their nearest, l = a
    # valid lower bound of the distance to every other previous centre
    dprev = torch.cdist(X[:, :d].double(), prevc.Cq[:k, :d].double())
    two = torch.topk(dprev, 2, dim=1, largest=False)
    a_prev = two.indices[:, 0].to(torch.int32)
    lold = (two.values[:, 1] * 0.999 - 1e-3).clamp_min(0).float()
    ul = torch.stack([two.values[:, 0].float() * 1.001 + 1e-3, lold], 1).contiguous()
    m = 60_001
    rows = torch.randperm(n, device=cuda)[:m].to(torch.int32)
    ws.acl[:m].copy_(a_prev[rows.long()])
    cnt = torch.tensor([m], dtype=torch.int64, device=cuda)
    K.sort_active(rows, cnt, ws)
    sel = torch.zeros(n, dtype=torch.bool, device=cuda)
    sel[rows.long()] = True
    a = torch.where(sel, a_prev, torch.full_like(a_prev, -7))
    changed = torch.empty(n, dtype=torch.int32, device=cuda)
    nch = torch.zeros(1, dtype=torch.int64, device=cuda)
    K.assign_rows(X, cen, ws.rows, n, a, post=dict(
        m_dev=cnt, a_prev=None, tol=tol, ul=ul, changed=changed, n_changed=nch,
        chg_new=torch.empty(n, dtype=torch.int32, device=cuda),
        chg_old=torch.empty(n, dtype=torch.int32, device=cuda)), cand=ws)
    assert bool((a[~sel] == -7).all())
    dist = torch.cdist(X[:, :d].double(), cen.Cq[:k, :d].double())
    bad = sel & (a != full)
    if bool(bad.any()):
        db = dist[bad].gather(1, a[bad].long()[:, None])[:, 0]
        df = dist[bad].gather(1, full[bad].long()[:, None])[:, 0]
        assert float(((db - df).abs() / df).max()) < 1e-4
    assert int(bad.sum()) <= (10 if tile16 else 5)   # near-ties (the gap check above)
    tw = torch.topk(dist, 2, dim=1, largest=False).values
    u, l = ul[:, 0], ul[:, 1]
    assert bool((u[sel].double() >= tw[sel, 0] - 1e-3).all())
    assert bool((l[sel].double() <= tw[sel, 1] + 1e-3).all())
    c = int(nch.item())
    exp = torch.nonzero(sel & (a != a_prev))[:, 0]
    assert c == exp.numel()
    assert torch.equal(torch.sort(changed[:c]).values.long(), exp)
