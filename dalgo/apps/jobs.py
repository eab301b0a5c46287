"""Reference-shaped benchmark jobs with correctness witnesses (BASELINE configs #4, #5).

Each function runs the reference script's whole JOB on this rank's share and returns a
dict (rank 0's view; clocks are the MAX over ranks):

* :func:`kmeans_job` -- machine_learning/k-means.py:53-71: takeSample-style init +
  ``n_iterations`` Lloyd iterations, iteration 1 (the full pass) inside the clock.
* :func:`pagerank_job` -- graph_computation/pagerank.py:41-57: the input edge list is
  given (generated before the clock, the ``parallelize(links)`` of :35-38); the clock
  covers ``distinct().groupByKey()`` + ``count()`` (relabel, dedup, adjacency / K4b
  layout build, out-degrees) and the 10 iterations. The process's caching allocator holds
  a device memory pool reserved before the clock (:func:`reserve_pool`).

Both are used by ``bench.py`` (secondary results of the driver's run) and by
``bench/kmeans_bench.py`` / ``bench/pagerank_bench.py``. A witness that fails sets
``passed: False`` in its record; the callers exit non-zero on it.
"""
from __future__ import annotations

import time

import torch

from dalgo.parallel import comm


def _max_over_ranks(x: float, device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    comm.all_reduce_max(t)
    return float(t.item())


class _Events:
    """HIP events between the phases of a job (no host sync inside the job)."""

    def __init__(self, device):
        self.cuda = device.type == "cuda"
        self.marks = []

    def mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append(e)
        else:
            self.marks.append(time.perf_counter())

    def spans(self):
        out = []
        for a, b in zip(self.marks[:-1], self.marks[1:]):
            out.append(a.elapsed_time(b) if self.cuda else (b - a) * 1e3)
        return out


def reserve_pool(device, gb: float) -> float:
    """Hold ``gb`` GiB (at most 80 % of the free memory) in the process's caching allocator:
    one allocation, freed at once, stays cached and later allocations are carved from it
    instead of going to hipMalloc (first-touch device allocations of hundreds of MB cost
    tens of ms each on ROCm). Done before a job's clock, like the memory pool a long-running
    job holds; returns the GiB reserved."""
    if device.type != "cuda" or gb <= 0:
        return 0.0
    free, _ = torch.cuda.mem_get_info(device)
    want = min(int(gb * (1 << 30)), int(free * 0.8))
    t = torch.empty(want, dtype=torch.uint8, device=device)
    del t
    return want / (1 << 30)


# --------------------------------------------------------------------- k-means
def kmeans_witness(km, rt) -> dict:
    """One more (untimed) iteration, checked against brute force from the same state:
    the assignment over the centres the step used differs from the full-pass K2 only at
    near-ties within the kernels' distance slack, the counts equal a K3 pass over it
    exactly and the maintained sums equal a full K3 pass."""
    from dalgo.ops import kmeans as K
    k, d = km.cfg.k, km.d
    cq = km.cen.Cq.clone()                     # the centres the next assignment uses
    km.step()
    rt.synchronize()
    cen_used = K.make_centers(cq[:k, :d].float(), km.X.dtype, rt.device, kpad=cq.shape[0])
    a_full = K.assign(km.X, cen_used)
    diff = (a_full != km.assign).nonzero().flatten()
    agree = 1.0 - diff.numel() / max(1, km.X.shape[0])
    Xd = km.X[diff, :d].double()
    Cd = cq[:k, :d].double()
    gap = ((Xd - Cd[km.assign[diff].long()]).pow(2).sum(1) -
           (Xd - Cd[a_full[diff].long()]).pow(2).sum(1)).abs()
    max_gap = float(gap.max().item()) if diff.numel() else 0.0
    # slack of a kernel distance: keys truncate 5 mantissa bits of 0.5|x-c|^2 + M
    xmax = 0.0
    for s0 in range(0, km.X.shape[0], 1 << 22):   # chunked: no 100M x 128 f32 temporary
        xmax = max(xmax, float((km.X[s0:s0 + (1 << 22), :d].float().pow(2).sum(1).max() * 0.5).item()))
    slack = 2.0 * (xmax * 1.0001 + 1e-6) * 2.0 ** -14 * 2.0
    S_ref = torch.zeros_like(km.S)
    c_ref = torch.zeros_like(km.cnt)
    K.accumulate(km.X, km.assign, k, km.DP, S_ref, c_ref)
    if km.incremental:
        S_m, c_m = km._S64, km._cnt64           # this rank's maintained local sums
    else:
        comm.all_reduce_sum(S_ref)              # the full path keeps only the global sums
        comm.all_reduce_sum(c_ref)
        S_m, c_m = km.S.double(), km.cnt
    err = float(((S_ref.double() - S_m.double()).abs().max() /
                 (1.0 + S_ref.double().abs().max())).item())
    counts_equal = bool(torch.equal(c_ref, c_m))
    ok = agree > 0.999 and max_gap <= slack and counts_equal and err < 1e-4
    okt = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=rt.device)
    comm.all_reduce_max(okt)
    return {"iteration": km.t, "path": "bounds" if km.bounds else (
                "incremental" if km.incremental else "full"),
            "assignment_agreement_vs_brute_force": agree, "disagreements": int(diff.numel()),
            "max_disagreement_gap": max_gap, "distance_slack": slack,
            "counts_equal": counts_equal, "sums_max_rel_err": err,
            "passed": bool(float(okt.item()) == 0.0)}


def kmeans_job(rt, rows: int = 100_000_000, dim: int = 128, k: int = 1024, iters: int = 5,
               dtype=torch.bfloat16, noise: float = 1.0, data_seed: int = 7,
               bound_filter: bool = True, candidates: bool = True, witness: bool = True,
               warm: bool = True, pool_gb: float = 48.0, dense: str = "auto", drift: bool = True) -> dict:
    """BASELINE config #4 (100M x 128, k = 1024): the reference's k-means job, strong
    scaling (the global point set is row-sharded over the ranks)."""
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.parallel.sharding import even_slices
    W = rt.world_size
    lo, hi = even_slices(rows, W)[rt.rank]
    reserve_pool(rt.device, pool_gb)
    if warm:
        # process warm-up (separate, small model; discarded): code objects and library
        # kernels loaded, as in any long-running job
        wn = min(1_000_000, rows)
        wlo, whi = even_slices(wn, W)[rt.rank]
        Xw = blobs(wn, dim, k, row_range=(wlo, whi), device=rt.device, dtype=dtype, seed=3,
                   noise=noise)
        kw = KMeans(KMeansConfig(k=min(k, wn), n_iterations=3, seed=5, bound_filter=bound_filter,
                                 candidates=candidates, dense=dense, drift=drift), Xw, wlo, wn)
        kw.step()
        kw.step()
        kw.step()
        del kw, Xw
    t0 = time.time()
    X = blobs(rows, dim, k, row_range=(lo, hi), device=rt.device, dtype=dtype, seed=data_seed,
              noise=noise)
    rt.synchronize()
    gen = time.time() - t0
    ev = _Events(rt.device)
    rt.barrier()
    rt.synchronize()
    t = time.perf_counter()
    ev.mark()
    km = KMeans(KMeansConfig(k=k, n_iterations=iters, seed=1, bound_filter=bound_filter,
                             candidates=candidates, dense=dense, drift=drift), X, lo, rows)
    ev.mark()
    for _ in range(iters):
        km.step()
        ev.mark()
    rt.synchronize()
    rt.barrier()
    rt.synchronize()
    job_ms = _max_over_ranks(time.perf_counter() - t, rt.device) * 1e3
    spans = ev.spans()
    init_ms, iter_ms = spans[0], spans[1:]
    sse_last = km.sse.clone()
    comm.all_reduce_sum(sse_last)
    active, moved, dense_rows = km.active_history, km.changed_history, km.dense_history
    wit = kmeans_witness(km, rt) if witness else None
    flops = 2.0 * rows * k * dim
    steady = iter_ms[1:]
    out = {
        "metric": "k-means points/sec (whole node)",
        "measured": f"reference job: init + {iters} Lloyd iterations, iteration 1 included",
        "value": rows * iters / (job_ms / 1e3), "unit": "points/s", "n_gpus": W,
        "job_ms": job_ms, "ms_per_iter": job_ms / iters, "iterations": iters,
        "init_ms_rank0": init_ms, "iteration_ms_rank0": iter_ms,
        "first_iteration_ms_rank0": iter_ms[0] if iter_ms else None,
        "steady_ms_per_iter_rank0": sum(steady) / len(steady) if steady else None,
        "full_pass_tflops_per_gpu": (flops / W / (iter_ms[0] / 1e3) / 1e12) if iter_ms else None,
        "reassigned_rows_per_iter_rank0": active, "moved_rows_per_iter_rank0": moved,
        "bound_filter": km.bounds, "candidate_pruning": getattr(km, "_cand", None) is not None,
        "dense_filtered_iterations": dense, "drift_pruned_candidates": drift,
        "dense_k2_rows_per_iter_rank0": dense_rows,
        "incremental_k3": km.incremental, "sse_last_iteration": float(sse_last.item()),
        "correctness_witness": wit,
        "config": {"rows": rows, "dim": dim, "k": k, "dtype": str(dtype).replace("torch.", ""),
                   "data": f"synthetic blobs (k Gaussians, spread 10, noise {noise})",
                   "init": "takeSample-style: k distinct seeded rows (k-means.py:53)"},
        "timing": "model construction + iterations 1..%d inside the clock (MAX over ranks); "
                  "process warmed up on a separate 1M-row model" % iters,
        "datagen_s": gen}
    del km, X
    return out


# --------------------------------------------------------------------- PageRank
def build_witness(edges: list, shard, pull_shard, rt) -> dict:
    """The adjacency build checked against torch over the RAW input edges (untimed), with
    nothing taken from the native keys: ``distinct()`` / ``count()`` of
    graph_computation/pagerank.py:41,44.

    * new_id is a bijection of [0, N);
    * this rank's distinct edges = torch.unique of the raw (src, dst) pairs relabelled
      through new_id and filtered to this rank's destinations: same count and the same
      edge set as the built shard (``pull_shard``, which the K4b-vs-pull check then uses);
    * the distinct out-degree of every local source (own slice and ghosts) = a bincount
      over that torch edge set, and the out-degrees sum to the edge count;
    * one rank: the distinct count of the un-relabelled input equals the built edge count
      (a bijective relabel preserves it).
    Every check is all-reduced (a failure on any rank fails the witness)."""
    dev = rt.device
    N, v_lo, v_hi, sl = shard.n_vertices, shard.v_lo, shard.v_hi, shard.slice_size
    nid = shard.new_id.long() if getattr(shard, "new_id", None) is not None else None
    bij = True
    if nid is not None:
        hit = torch.zeros(N, dtype=torch.int32, device=dev)
        hit.index_fill_(0, nid, 1)
        bij = bool(int(nid.min().item()) >= 0 and int(nid.max().item()) < N and int(hit.sum().item()) == N)
        del hit
    parts = []
    raw_parts = []
    for s, d in edges:
        s64, d64 = s.long(), d.long()
        if rt.world_size == 1:
            raw_parts.append((s64 << 32) | d64)
        if nid is not None:
            s64, d64 = nid[s64], nid[d64]
        keep = (d64 >= v_lo) & (d64 < v_hi)
        parts.append(((d64[keep] - v_lo) << 32) | s64[keep])
        del s64, d64, keep
    ref = torch.unique(torch.cat(parts))
    del parts
    n_ref = int(ref.numel())
    raw_distinct = None
    if raw_parts:
        raw_distinct = int(torch.unique(torch.cat(raw_parts)).numel())
    del raw_parts
    E = pull_shard.n_edges
    got = (pull_shard.dstl[:E].long() << 32) | pull_shard.src[:E].long()
    same_set = n_ref == E and bool(torch.equal(got, ref))
    del got
    # distinct out-degree per local source (the [own | ghost] index space of the native build)
    od_ok = True
    od = getattr(shard, "outdeg_loc", None)
    if od is not None:
        src = ref & 0xFFFFFFFF
        own = (src >= v_lo) & (src < v_hi)
        cnt = torch.zeros(od.numel(), dtype=torch.int64, device=dev)
        cnt.index_add_(0, src[own] - v_lo, torch.ones_like(src[own]))
        gh = getattr(shard, "ghosts", None)
        if gh is not None and gh.numel():
            gi = torch.searchsorted(gh, src[~own])
            ok_g = bool((gi < gh.numel()).all().item()) and bool(torch.equal(gh[gi.clamp_max(gh.numel() - 1)], src[~own]))
            od_ok = ok_g
            cnt.index_add_(0, sl + gi.clamp_max(gh.numel() - 1), torch.ones_like(gi))
        od_ok = od_ok and bool(torch.equal(cnt, od.long())) and int(od.long().sum().item()) == E
        del src, own, cnt
    del ref
    ok = bij and same_set and od_ok and (raw_distinct is None or raw_distinct == E)
    okt = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=dev)
    comm.all_reduce_max(okt)
    return {"vs": "torch.unique over the raw input edges (relabelled through new_id)",
            "relabel_bijective": bij, "edges_rank0": E, "torch_distinct_rank0": n_ref,
            "edge_set_equal_rank0": same_set, "outdeg_equal_rank0": od_ok,
            "raw_distinct_one_rank": raw_distinct,
            "passed": bool(float(okt.item()) == 0.0)}


def pagerank_job(rt, scale: int = 26, edge_factor: int = 16, iters: int = 10,
                 spmv: str = "blocked", semantics: str = "reference", witness: bool = True,
                 reorder: bool = True, seed: int = 1, bin_width: int = 16384,
                 chunk: int = 1 << 40, tile: int = 16384, timed_iters: int = 10,
                 native_build: bool = True, pool_gb: float = 96.0, warm: bool = True) -> dict:
    """BASELINE config #5 (R-MAT scale 26, edge factor 16 = 1.07B edges, Graph500
    a,b,c = 0.57,0.19,0.19, scrambled ids): the reference's PageRank job, destination-
    partitioned over the ranks. The input edge list is generated before the clock; the
    clock covers the adjacency build (degree relabeling, dedup, out-degrees, K4b layout)
    plus ``iters`` iterations. After it, ``timed_iters`` more iterations are timed alone
    (per-iteration edges/s, secondary) and the witness checks one more K4b step against
    the pull K4 SpMV from the same state. ``warm``: the same build + 2 iterations on a
    separate scale-16 graph first (discarded), as the k-means job does: the first launch of
    every library kernel loads its code object (tens of ms each on a cold process)."""
    from dalgo.apps.pagerank_app import (build_rmat_native, build_rmat_shard, build_rmat_sharded,
                                         rmat_input, rmat_input_share)
    from dalgo.models.pagerank import PageRank, PageRankConfig
    from dalgo.utils.obs import PhaseTimer
    W = rt.world_size
    pool = reserve_pool(rt.device, pool_gb)
    native = (native_build and rt.device.type == "cuda" and spmv == "blocked" and chunk >= 1 << 40)
    # several ranks: every rank holds E / W input edges and the build shuffles them to
    # their destination owners (pagerank_app.build_rmat_sharded); one rank: the whole
    # stream through the packed one-rank build
    sharded = W > 1
    cfg = PageRankConfig(semantics=semantics, spmv=spmv, bin_width=bin_width, chunk=chunk,
                         tile=tile, n_iterations=iters)
    if warm:
        ws = min(16, scale)
        if sharded:
            we, _ = rmat_input_share(ws, edge_factor, rt.rank, W, rt.device, seed + 1)
        else:
            we, _ = rmat_input(ws, edge_factor, rt.device, seed + 1)
        if sharded:
            wsh = build_rmat_sharded(we, ws, rt.rank, W, rt.device, reorder=reorder, native=native,
                                     keep_keys=witness, bin_width=bin_width, tile=tile)
        elif native:
            wsh = build_rmat_native(we, ws, rt.rank, W, rt.device, reorder=reorder, keep_keys=witness,
                                    bin_width=bin_width, tile=tile)
        else:
            wsh = build_rmat_shard(we, ws, rt.rank, W, rt.device, reorder=reorder, seed=seed)
        wpr = PageRank(cfg, wsh, W)
        wpr.step()
        wpr.step()
        rt.synchronize()
        del we, wsh, wpr
    t0 = time.time()
    if sharded:
        edges, n_gen = rmat_input_share(scale, edge_factor, rt.rank, W, rt.device, seed)
    else:
        edges, n_gen = rmat_input(scale, edge_factor, rt.device, seed)
    rt.synchronize()
    gen_s = time.time() - t0
    ev = _Events(rt.device)
    rt.barrier()
    rt.synchronize()
    t = time.perf_counter()
    ev.mark()
    # GPU + blocked SpMV + (one rank or the ghost exchange): the native build straight into
    # the K4b layout; otherwise the (dst, src)-sorted shard
    if native:
        from dalgo.ops import graph as G
        G.build_marks = []
    if sharded:
        shard = build_rmat_sharded(edges, scale, rt.rank, W, rt.device, reorder=reorder, native=native,
                                   keep_keys=witness, bin_width=bin_width, tile=tile)
    elif native:
        shard = build_rmat_native(edges, scale, rt.rank, W, rt.device, reorder=reorder,
                                  keep_keys=witness, bin_width=bin_width, tile=tile)
    else:
        shard = build_rmat_shard(edges, scale, rt.rank, W, rt.device, reorder=reorder, seed=seed)
    ev.mark()
    pr = PageRank(cfg, shard, W)
    ev.mark()
    for _ in range(iters):
        pr.step()
    ev.mark()
    rt.synchronize()
    rt.barrier()
    rt.synchronize()
    job_ms = _max_over_ranks(time.perf_counter() - t, rt.device) * 1e3
    shard_ms, model_ms, iters_ms = ev.spans()
    build_phases = None
    if native:
        from dalgo.ops import graph as G
        build_phases = G.build_phase_spans()
        G.build_marks = None
    E = comm.all_reduce_count(shard.n_edges, device=rt.device)
    # per-iteration rate alone (after the job), with the phase split of one step
    pr.timer = PhaseTimer(rt.device)
    pr.step()
    rt.synchronize()
    phases = pr.timer.summary()
    pr.timer = None
    rt.barrier()
    rt.synchronize()
    t = time.perf_counter()
    for _ in range(timed_iters):
        pr.step()
    rt.synchronize()
    rt.barrier()
    rt.synchronize()
    it_ms = _max_over_ranks(time.perf_counter() - t, rt.device) / max(timed_iters, 1) * 1e3
    wit = None
    bwit = None
    pull_shard = None
    if witness:
        pull_shard = shard.to_shard() if native else shard
        if sharded:   # the witness needs every input edge: the same stream, regenerated
            del edges
            edges, _ = rmat_input(scale, edge_factor, rt.device, seed)
        bwit = build_witness(edges, shard, pull_shard, rt)
    del edges
    if witness:
        # one more iteration of the benchmarked SpMV vs the pull SpMV from the same state
        ref = PageRank(PageRankConfig(semantics=semantics, spmv="pull", exchange=pr.exchange),
                       pull_shard, W)
        ref.load_state_dict(pr.state_dict())
        pr.step()
        ref.step()
        rt.synchronize()
        r1, r0 = pr.r.double(), ref.r.double()
        both = (r1 >= 0) & (r0 >= 0)
        err = torch.tensor([float(((r1 - r0).abs() * both).max().item()) if r1.numel() else 0.0,
                            float((r1 >= 0).ne(r0 >= 0).sum().item())], dtype=torch.float64,
                           device=rt.device)
        comm.all_reduce_max(err)
        sc = torch.tensor([float(r0.abs().max().item()) if r0.numel() else 0.0],
                          dtype=torch.float64, device=rt.device)
        comm.all_reduce_max(sc)
        rel = float(err[0].item()) / max(float(sc.item()), 1e-30)
        wit = {"vs": "pull K4 SpMV, same state", "max_rel_err": rel,
               "presence_mismatches": int(err[1].item()), "iteration": pr.t,
               "build": bwit,
               "passed": bool(rel < 1e-5 and int(err[1].item()) == 0 and bwit["passed"])}
        del ref, pull_shard
    lay = pr.layout
    out = {
        "metric": "PageRank edges/sec (whole node)",
        "measured": f"reference job: adjacency build (relabel, dedup, degrees, layout) + "
                    f"{iters} iterations",
        "value": E * iters / (job_ms / 1e3), "unit": "edges/s", "n_gpus": W,
        "job_ms": job_ms, "build_ms_rank0": shard_ms + model_ms,
        "shard_build_ms_rank0": shard_ms, "model_build_ms_rank0": model_ms,
        "build_phases_ms_rank0": build_phases,
        "iterations_ms_rank0": iters_ms,
        "ms_per_iter": it_ms, "edges_per_s_per_iter": E / (it_ms / 1e3),
        "edges_dedup": E, "edges_generated": n_gen, "vertices": 1 << scale,
        "degree_reordered": reorder, "spmv": pr.spmv, "exchange": pr.exchange,
        "adjacency_build": ("native (graph_build.hip)" if native else "torch (dst, src) shard") + (
            ", sharded input (E / W edges per rank, all_to_all to the destination owners)"
            if sharded else ""),
        "phases_ms_rank0": phases, "correctness_witness": wit,
        "allocator_pool_gib": pool,
        "timing": "adjacency build + %d iterations inside the clock (MAX over ranks); input "
                  "edges generated before it; %s" % (iters, "process warmed up on a separate "
                  "scale-%d graph" % min(16, scale) if warm else "cold process"),
        "blocked_layout_rank0": None if lay is None else {
            "chunks": lay.n_chunks, "entries": lay.n_entries,
            "entries_per_edge": lay.n_entries / max(shard.n_edges, 1),
            "work_items": int(lay.wi_bin.numel()), "split_bins": int(lay.split_bin.numel()),
            "bin_width": lay.bin_width},
        "config": {"scale": scale, "edge_factor": edge_factor, "semantics": semantics,
                   "data": "synthetic Graph500 R-MAT (0.57, 0.19, 0.19), scrambled ids"},
        "datagen_s": gen_s}
    del pr, shard
    return out
