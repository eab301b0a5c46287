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
    a = ap.parse_args()
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.ops import kmeans as K
    from dalgo.parallel import comm, runtime
    from dalgo.parallel.sharding import even_slices
    rt = runtime.init(device="cuda")
    W = rt.world_size
    lo, hi = even_slices(a.rows, W)[rt.rank]
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    t0 = time.time()
    X = blobs(a.rows, a.dim, a.k, row_range=(lo, hi), device=rt.device, dtype=dtype, seed=7)
    torch.cuda.synchronize()
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
    torch.cuda.synchronize()
    rt.barrier(); torch.cuda.synchronize()
    km.timer = PhaseTimer(rt.device)     # HIP events only (no host sync in the loop)
    km.changed_history.clear()
    km.active_history.clear()
    t = time.perf_counter()
    for _ in range(a.steps):
        km.step()
    torch.cuda.synchronize(); rt.barrier(); torch.cuda.synchronize()
    timed_phases = {k: v / a.steps for k, v in km.timer.summary().items()}
    phases = first or {}
    sse_last = km.sse.clone()
    comm.all_reduce_sum(sse_last)
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=rt.device)
    comm.all_reduce_max(el)
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
            "accumulate_mode": "incremental below %.1f %% moved rows" % (100 * km.inc_max)
            if km.inc_max > 0 else "full", "config": {"rows": a.rows, "dim": a.dim, "k": a.k, "dtype": a.dtype},
            "datagen_s": gen}), flush=True)
    runtime.shutdown()


if __name__ == "__main__":
    main()
