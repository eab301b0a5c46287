#!/usr/bin/env python3
"""K-means benchmark (BASELINE config: 100M x 128, k=1024, bf16).

Strong scaling: the global N x d point set is row-sharded over the ranks.
Reports points/s (whole job), per-phase times and the achieved TFLOP/s of the
fused distance GEMM (2*N*k*d FLOP per iteration).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="ranks (one per GPU); started here as a torchrun child when > 1")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"])
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    from dalgo.parallel.launch import check_world, self_launch
    rc = self_launch(a.gpus, __file__, argv, device=a.device, backend=a.backend, tag="kmeans_bench")
    if rc is not None:
        sys.exit(rc)
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.ops import kmeans as K
    from dalgo.parallel import comm, runtime
    from dalgo.parallel.sharding import even_slices
    rt = runtime.init(backend=a.backend, device=a.device, app_name="kmeans-bench")
    W = rt.world_size
    check_world(a.gpus, W, "kmeans_bench")
    lo, hi = even_slices(a.rows, W)[rt.rank]
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    t0 = time.time()
    X = blobs(a.rows, a.dim, a.k, row_range=(lo, hi), device=rt.device, dtype=dtype, seed=7)
    rt.synchronize()
    gen = time.time() - t0
    km = KMeans(KMeansConfig(k=a.k, n_iterations=a.steps, seed=1), X, lo, a.rows)
    from dalgo.utils.obs import PhaseTimer
    # warmup: the first iteration is the full pass (full K2 + K3, bounds built); its
    # phases are reported separately
    km.timer = PhaseTimer(rt.device)
    first = None
    for i in range(a.warmup):
        km.step()
        if i == 0:
            first = km.timer.summary()
            km.timer = PhaseTimer(rt.device)
    rt.synchronize()
    rt.barrier(); rt.synchronize()
    km.timer = PhaseTimer(rt.device)     # HIP events only (no host sync in the loop)
    km.changed_history.clear()
    km.active_history.clear()
    t = time.perf_counter()
    for _ in range(a.steps):
        km.step()
    rt.synchronize(); rt.barrier(); rt.synchronize()
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=rt.device)
    comm.all_reduce_max(el)
    timed_phases = {k: v / a.steps for k, v in km.timer.summary().items()}
    phases = first or {}
    sse_last = km.sse.clone()
    comm.all_reduce_sum(sse_last)
    # correctness witness (untimed): the last assignment vs a brute-force K2 pass over all
    # points with the same (rounded) centres, and the incrementally maintained local sums /
    # counts vs a full K3 pass over that assignment
    witness = None
    if km.bounds and km._u is not None:
        d = km.d
        cen_last = K.make_centers(km._cq_prev[:, :d].float(), km.X.dtype, rt.device,
                                  kpad=km.cen.Cq.shape[0])
        sse_bf = torch.zeros(1, dtype=torch.float32, device=rt.device)
        a_full = K.assign(km.X, cen_last, sse=sse_bf)
        if isinstance(a_full, tuple):
            a_full = a_full[0]
        diff = (a_full != km.assign).nonzero().flatten()
        agree = 1.0 - diff.numel() / max(1, km.X.shape[0])
        # every disagreement must be a near-tie: both centres within the kernel's
        # distance slack of each other (exact f64 distances on the rounded centres)
        Xd = km.X[diff, :d].double()
        Cd = km._cq_prev[:, :d].double()
        gap = ((Xd - Cd[km.assign[diff].long()]).pow(2).sum(1) -
               (Xd - Cd[a_full[diff].long()]).pow(2).sum(1)).abs()
        max_gap = float(gap.max().item()) if diff.numel() else 0.0
        S_ref = torch.zeros_like(km.S)
        c_ref = torch.zeros_like(km.cnt)
        K.accumulate(km.X, km.assign, a.k, km.DP, S_ref, c_ref)
        err = float(((S_ref.double() - km._S64).abs().max() /
                     (1.0 + S_ref.double().abs().max())).item())
        witness = {"assignment_agreement_vs_brute_force": agree,
                   "disagreements": int(diff.numel()),
                   "max_disagreement_gap": max_gap, "distance_slack": 2.0 * km._tol,
                   "counts_equal": bool(torch.equal(c_ref, km._cnt64)),
                   "sums_max_rel_err": err,
                   "local_sse_identity_vs_kernel_rel": float(
                       ((km.sse.double() - sse_bf.double()).abs() /
                        sse_bf.double().abs().clamp_min(1e-30)).item()),
                   "passed": bool(agree > 0.999 and max_gap <= 2.0 * km._tol and torch.equal(c_ref, km._cnt64) and err < 1e-4)}
    ms = float(el.item()) / a.steps * 1e3
    flops = 2.0 * a.rows * a.k * a.dim
    if rt.is_main:
        print(json.dumps({
            "metric": "k-means points/sec (whole node)", "value": a.rows / (ms / 1e3), "unit": "points/s",
            "n_gpus": W, "ms_per_iter": ms, "full_assign_tflops_per_gpu": flops / W / (phases["assign"] / 1e3) / 1e12 if phases.get("assign") else None,
            "first_iteration_phases_ms_rank0": phases,
            "timed_phases_ms_per_iter_rank0": timed_phases,
            "moved_rows_per_iter_rank0": list(km.changed_history),
            "reassigned_rows_per_iter_rank0": list(km.active_history),
            "bound_filter": km.bounds, "sse_last_iteration": float(sse_last.item()),
            "correctness_witness": witness,
            "accumulate_mode": "incremental below %.1f %% moved rows" % (100 * km.inc_max)
            if km.inc_max > 0 and km.X.is_cuda else "full", "config": {"rows": a.rows, "dim": a.dim, "k": a.k, "dtype": a.dtype},
            "datagen_s": gen}), flush=True)
    runtime.shutdown()


if __name__ == "__main__":
    main()
