"""Multi-rank (gloo, world_size=2) == single-rank equivalence for every algorithm."""
import math

import numpy as np
import pytest
import torch

from tests.dist_util import run_world


def _lr_family(rt):
    from dalgo.data.datasets import breast_cancer
    from dalgo.models.localsgd import ParallelSGD, SGDConfig
    from dalgo.parallel.sharding import make_layout
    out = {}
    for algo in ("ssgd", "gd", "ma", "bmuf", "easgd"):
        cfg = SGDConfig(algo=algo, n_iterations=12, eval_every=0)
        lay = make_layout(398, cfg.n_workers, rt.world_size, rt.rank)
        d = breast_cancer(dtype=torch.float64, row_range=(lay.row_lo, lay.row_hi))
        m = ParallelSGD(cfg, d, lay, rt, model_dtype=torch.float64)
        m.fit()
        out[algo] = m.weights().numpy().copy()
    return out


def _others(rt):
    from dalgo.models.als import ALS, ALSConfig
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.models.monte_carlo import MonteCarloConfig, estimate_pi
    from dalgo.models.pagerank import PageRank, PageRankConfig
    from dalgo.models.transitive_closure import DenseClosure, SparseClosure
    from dalgo.data.synthetic import blobs
    from dalgo.ops import graph as G
    from dalgo.parallel.sharding import even_slices
    W, r = rt.world_size, rt.rank
    out = {}
    # k-means on blobs
    n = 3000
    lo, hi = even_slices(n, W)[r]
    X = blobs(n, 5, 4, row_range=(lo, hi), seed=3)
    km = KMeans(KMeansConfig(k=4, n_iterations=4, seed=1), X, lo, n)
    km.fit()
    out["kmeans"] = km.centers.numpy().copy()
    out["kmeans_sse"] = km.history.sse
    # pagerank on a small R-MAT graph, both semantics
    s, d = G.rmat_edges(6000, 10, seed=9)
    for sem in ("reference", "standard"):
        sh = G.build_shard(s, d, 1024, r, W)
        out["pr_" + sem] = PageRank(PageRankConfig(semantics=sem), sh, W).fit().collect()
        # the all_gather exchange (the default on several ranks is the ghost exchange)
        out["pr_ag_" + sem] = PageRank(PageRankConfig(semantics=sem, exchange="allgather"), sh,
                                       W).fit().collect()
        # K4b propagation-blocked SpMV over the ghost index space
        out["pr_pb_" + sem] = PageRank(PageRankConfig(semantics=sem, spmv="blocked", chunk=256,
                                                      tile=64), sh, W).fit().collect()
    # transitive closure
    g = torch.Generator().manual_seed(4)
    ts = torch.randint(0, 60, (100,), generator=g)
    td = torch.randint(0, 60, (100,), generator=g)
    out["tc_dense"] = DenseClosure(ts, td, 60, r, W).run().counts
    out["tc_sparse"] = SparseClosure(ts, td, r, W, n=60).run().counts
    # ALS
    out["als"] = ALS(ALSConfig(m=40, n=60, k=5, seed=2), r, W).fit().rmse
    # Monte Carlo
    out["mc"] = estimate_pi(MonteCarloConfig(n=200_000), r, W)
    return out


@pytest.fixture(scope="module")
def lr_results():
    one = run_world(_lr_family, world=1)[0]
    two = run_world(_lr_family, world=2)
    return one, two


@pytest.mark.parametrize("algo", ["ssgd", "gd", "ma", "bmuf", "easgd"])
def test_lr_family_two_ranks_equal_one(lr_results, algo):
    one, two = lr_results
    assert np.allclose(two[0][algo], two[1][algo], rtol=0, atol=0)        # replicated state
    ref = one[algo]
    assert np.allclose(two[0][algo], ref, rtol=1e-10, atol=1e-8 * max(1, np.abs(ref).max()))


def test_other_algorithms_two_ranks_equal_one():
    one = run_world(_others, world=1)[0]
    two = run_world(_others, world=2)
    for k in ("kmeans",):
        assert np.allclose(two[0][k], one[k], atol=1e-4), k
        assert np.allclose(two[1][k], one[k], atol=1e-4), k
    assert np.allclose(two[0]["kmeans_sse"], one["kmeans_sse"], rtol=1e-6)
    for sem in ("pr_reference", "pr_standard", "pr_ag_reference", "pr_ag_standard",
                "pr_pb_reference", "pr_pb_standard"):
        a, b = one[sem], two[0][sem]
        assert set(a) == set(b)
        assert max(abs(a[v] - b[v]) for v in a) < 1e-12
        assert b == two[1][sem]
    assert one["tc_dense"] == two[0]["tc_dense"] == one["tc_sparse"] == two[1]["tc_sparse"]
    assert np.allclose(one["als"], two[0]["als"], rtol=1e-9)
    assert one["mc"] == two[0]["mc"] == two[1]["mc"]
    assert abs(one["mc"][0] - math.pi) < 0.02


def _pr_peer(rt):
    """K4b with the ghost exchange run as W - 1 per-peer shifts (each peer's ghost chunks
    consumed as its shift lands) vs the whole all_to_all and vs no overlap."""
    from dalgo.models.pagerank import PageRank, PageRankConfig
    from dalgo.ops import graph as G
    W, r = rt.world_size, rt.rank
    s, d = G.rmat_edges(6000, 10, seed=5)
    out = {}
    for sem in ("reference", "standard"):
        sh = G.build_shard(s, d, 1024, r, W)
        for ov in ("peer", "on", "off"):
            pr = PageRank(PageRankConfig(semantics=sem, spmv="blocked", chunk=256, tile=64,
                                         overlap=ov), sh, W)
            out[(sem, ov, "mode")] = pr._overlap_pb()
            out[(sem, ov)] = pr.fit().collect()
    return out


def test_pagerank_per_peer_overlap_three_ranks():
    one = run_world(_pr_peer, world=1)[0]
    three = run_world(_pr_peer, world=3)
    for sem in ("reference", "standard"):
        assert three[0][(sem, "peer", "mode")] == "peer"
        ref = one[(sem, "off")]
        for ov in ("peer", "on", "off"):
            got = three[0][(sem, ov)]
            assert set(got) == set(ref)
            assert max(abs(got[v] - ref[v]) for v in ref) < 1e-12, (sem, ov)


def _error_check_body(rt):
    """Rank 1 alone carries a set K11 error word; both ranks must raise."""
    import torch

    from dalgo.parallel import comm, xgmi

    class _Fake:
        err = torch.ones(1, dtype=torch.int32) if rt.rank == 1 else torch.zeros(1, dtype=torch.int32)

    xgmi._shared["fake"] = _Fake()
    raised = False
    try:
        comm.check_device_errors("test")
    except comm.DeviceCollectiveError:
        raised = True
    finally:
        del xgmi._shared["fake"]
        comm._error_seen = False      # let the harness' shutdown exit cleanly
    # clean words: no raise on any rank
    comm.check_device_errors("test-clean")
    return raised


def test_device_error_check_raises_on_every_rank():
    """a peer-wait timeout on ONE rank raises on EVERY rank (collective MAX
    first), so no rank is left blocked in a later collective."""
    assert run_world(_error_check_body, world=2) == [True, True]


def test_other_algorithms_three_ranks_equal_one():
    """Odd world size: uneven vertex / row / factor slices (3000 points, 1024-vertex
    slices of a 6000-vertex graph, 40 / 60 ALS rows over 3 ranks)."""
    one = run_world(_others, world=1)[0]
    three = run_world(_others, world=3)
    for r in range(3):
        assert np.allclose(three[r]["kmeans"], one["kmeans"], atol=1e-4), r
        assert three[r]["tc_dense"] == one["tc_dense"] == three[r]["tc_sparse"]
        assert three[r]["mc"] == three[0]["mc"]
    assert np.allclose(three[0]["kmeans_sse"], one["kmeans_sse"], rtol=1e-6)
    for sem in ("pr_reference", "pr_standard", "pr_ag_reference", "pr_ag_standard"):
        a, b = one[sem], three[0][sem]
        assert set(a) == set(b)
        assert max(abs(a[v] - b[v]) for v in a) < 1e-12
        assert b == three[1][sem] == three[2][sem]
    assert np.allclose(one["als"], three[0]["als"], rtol=1e-9)


def _lr_four(rt):
    return _lr_family(rt)


def test_lr_family_four_ranks_equal_one(lr_results):
    """One logical worker (Spark partition) per rank: P = W = 4."""
    one, _ = lr_results
    four = run_world(_lr_four, world=4)
    for algo in ("ssgd", "gd", "ma", "bmuf", "easgd"):
        ref = one[algo]
        for r in range(4):
            assert np.allclose(four[r][algo], ref, rtol=1e-10,
                               atol=1e-8 * max(1, np.abs(ref).max())), (algo, r)


def _comm_body(rt):
    import torch

    from dalgo.parallel import comm
    W, r = rt.world_size, rt.rank
    out = {}
    x = torch.arange(5, dtype=torch.float64) * (r + 1)
    comm.all_reduce_sum(x)
    out["sum"] = x.tolist()
    m = torch.tensor([float(r * 7 % 5)], dtype=torch.float64)
    comm.all_reduce_max(m)
    out["max"] = float(m.item())
    out["count"] = comm.all_reduce_count(r + 2)
    b = torch.full((3,), float(r), dtype=torch.float64)
    comm.broadcast(b, src=W - 1)
    out["bcast"] = b.tolist()
    full = torch.empty(2 * W, dtype=torch.float64)
    comm.all_gather_into(full, torch.tensor([r, 10 * r], dtype=torch.float64))
    out["gather"] = full.tolist()
    counts = [i + 1 for i in range(W)]                       # uneven: 1, 2, 3 rows
    loc = torch.full((counts[r], 2), float(r), dtype=torch.float64)
    out["varlen"] = comm.all_gather_varlen(loc, counts).tolist()
    rs = torch.empty(2, dtype=torch.float64)
    comm.reduce_scatter_sum(rs, torch.arange(2 * W, dtype=torch.float64) + r)
    out["rs"] = rs.tolist()
    g0 = comm.gather_to_rank0(torch.full((counts[r],), float(r), dtype=torch.float64), counts)
    out["g0"] = None if g0 is None else g0.tolist()
    bk = comm.BucketedAllReduce([(2, 3), (1,)], dtype=torch.float64, device=torch.device("cpu"))
    a, c = bk.views
    a.fill_(float(r))
    c.fill_(1.0)
    bk.all_reduce()
    out["bucket"] = (a.tolist(), c.tolist())
    return out


def test_comm_primitives_three_ranks():
    W = 3
    res = run_world(_comm_body, world=W)
    for r, o in enumerate(res):
        assert o["sum"] == [i * 6.0 for i in range(5)]
        assert o["max"] == 4.0                                # 0, 7 % 5 = 2, 14 % 5 = 4
        assert o["count"] == 2 + 3 + 4
        assert o["bcast"] == [2.0, 2.0, 2.0]
        assert o["gather"] == [0.0, 0.0, 1.0, 10.0, 2.0, 20.0]
        assert o["varlen"] == [[0.0, 0.0]] + [[1.0, 1.0]] * 2 + [[2.0, 2.0]] * 3
        assert o["rs"] == [float(3 * (2 * r) + 3), float(3 * (2 * r + 1) + 3)]
        assert o["bucket"] == ([[3.0] * 3] * 2, [3.0])
        if r == 0:
            assert o["g0"] == [0.0, 1.0, 1.0, 2.0, 2.0, 2.0]
        else:
            assert o["g0"] is None


def _easgd_overlap(rt):
    from dalgo.data.datasets import breast_cancer
    from dalgo.models.localsgd import ParallelSGD, SGDConfig
    from dalgo.parallel.sharding import make_layout
    out = {}
    for ov in (True, False):
        cfg = SGDConfig(algo="easgd", n_iterations=15, eval_every=4, overlap_center=ov)
        lay = make_layout(398, cfg.n_workers, rt.world_size, rt.rank)
        d = breast_cancer(dtype=torch.float64, row_range=(lay.row_lo, lay.row_hi))
        m = ParallelSGD(cfg, d, lay, rt, model_dtype=torch.float64)
        h = m.fit()
        out[ov] = (m.weights().numpy().copy(), list(h.accs), m.state_dict()["w"].numpy().copy())
    return out


def test_easgd_centre_overlap_is_exact():
    """The deferred (overlapped) EASGD centre all-reduce computes exactly the sequential
    rounds of easgd.py:95-106: same weights, same evaluation history, same checkpoint."""
    for res in run_world(_easgd_overlap, world=2):
        a, b = res[True], res[False]
        assert np.array_equal(a[0], b[0])
        assert a[1] == b[1]
        assert np.array_equal(a[2], b[2])


def _easgd_overlap_rules(rt):
    """EASGD's deferred centre all-reduce is never used under hipGraph replay: a captured
    step must not consume a collective issued outside the graph."""
    from dalgo.data.datasets import breast_cancer
    from dalgo.models.localsgd import ParallelSGD, SGDConfig
    from dalgo.parallel.sharding import make_layout
    cfg = SGDConfig(algo="easgd", n_iterations=4, eval_every=0)
    lay = make_layout(398, cfg.n_workers, rt.world_size, rt.rank)
    d = breast_cancer(dtype=torch.float64, row_range=(lay.row_lo, lay.row_hi))
    m = ParallelSGD(cfg, d, lay, rt, model_dtype=torch.float64)
    eager = m._overlap_ok()
    m._okg = True          # as if graph replay had been selected
    graphed = m._overlap_ok()
    return eager, graphed


def test_easgd_overlap_off_under_graph_replay():
    res = run_world(_easgd_overlap_rules, world=2)
    assert all(r == (True, False) for r in res)


def _kmeans_big_counts(rt):
    """The fused [S || count pairs] bucket is exact for counts beyond 2^24 per rank."""
    from dalgo.models.kmeans import KMeans, KMeansConfig
    X = torch.zeros((8, 2))
    X[4:, 0] = 1.0
    km = KMeans(KMeansConfig(k=2, n_iterations=1), X, 8 * rt.rank, 8 * rt.world_size,
                init_centers=torch.tensor([[0.0, 0.0], [1.0, 0.0]]))
    from dalgo.ops import kmeans as K
    orig = K.accumulate

    def fake(Xp, a, k, DP, S, cnt, method="sorted"):
        orig(Xp, a, k, DP, S, cnt)
        cnt += (1 << 25) + 12345 * (rt.rank + 1)   # pretend huge clusters
        return S, cnt
    K.accumulate = fake
    try:
        km.step()
    finally:
        K.accumulate = orig
    return km.cnt.tolist()


def test_kmeans_fused_bucket_exact_large_counts():
    res = run_world(_kmeans_big_counts, world=3)
    extra = 3 * (1 << 25) + 12345 * 6
    assert all(r == [12 + extra, 12 + extra] for r in res), res


def _pr_sharded(rt, scale):
    """Sharded-input build (each rank E / W edges, shuffle to destination owners) vs the
    full-stream build of the same rank with the same relabeling; PageRank ranks in the
    generator's ids."""
    from dalgo.apps.pagerank_app import (build_rmat_sharded, build_rmat_shard, rmat_input,
                                         rmat_input_share)
    from dalgo.models.pagerank import PageRank, PageRankConfig
    W, r = rt.world_size, rt.rank
    mine, n_e = rmat_input_share(scale, 8, r, W, "cpu", seed=3)
    sh = build_rmat_sharded(mine, scale, r, W, "cpu", reorder=True)
    full, _ = rmat_input(scale, 8, "cpu", seed=3, chunk=1 << 11)
    ref = build_rmat_shard(full, scale, r, W, "cpu", reorder=True)
    E = sh.n_edges
    got = (sh.dstl[:E].long() << 32) | sh.src[:E].long()
    exp = (ref.dstl[:ref.n_edges].long() << 32) | ref.src[:ref.n_edges].long()
    pr = PageRank(PageRankConfig(), sh, W).fit()
    ranks = pr.collect()
    inv = torch.empty_like(sh.new_id, dtype=torch.int64)
    inv[sh.new_id.long()] = torch.arange(sh.new_id.numel())
    return {"same_new_id": bool(torch.equal(sh.new_id.long(), ref.new_id.long())),
            "same_edges": bool(torch.equal(got, exp)), "E": E,
            "ranks": {int(inv[v]): x for v, x in ranks.items()}}


@pytest.mark.parametrize("world", [2, 3])
def test_pagerank_sharded_input_build(world):
    scale = 11
    res = run_world(_pr_sharded, world=world, args=(scale,))
    one = run_world(_pr_sharded, world=1, args=(scale,))[0]
    for r in res:
        assert r["same_new_id"] and r["same_edges"]
    assert sum(r["E"] for r in res) == one["E"]
    for r in res:
        for v, x in r["ranks"].items():
            assert math.isclose(x, one["ranks"][v], rel_tol=1e-9, abs_tol=1e-15)
    assert set(res[0]["ranks"]) == set(one["ranks"])
