#!/usr/bin/env python3
"""K-means benchmark (BASELINE config #4: 100M x 128, k = 1024, bf16).

Headline = the reference's JOB (machine_learning/k-means.py:18,53-71): the model is
built from a takeSample-style init (k distinct seeded rows) and runs n_iterations = 5
Lloyd iterations; the clock covers model construction + all 5 iterations, iteration 1
(the full pass) included -- no untimed warm-up iteration of the model. Before it, the
PROCESS is warmed up once on a separate small problem (1M rows, same d / k, two
iterations) so GPU code objects and library kernels are loaded, as in any long-running
job; that model is discarded. Per-iteration device times come from HIP events recorded
between the iterations (no host sync inside the loop); iterations 2.. are reported as
``steady_ms_per_iter`` (secondary).

Strong scaling: the global N x d point set is row-sharded over the ranks; the clock is
the MAX over ranks. A correctness witness runs after the timed job (untimed): one more
iteration, whose assignment must agree with a brute-force K2 pass over the centres it
used (every disagreement a near-tie within the kernel's distance slack) and whose
incrementally maintained local sums / counts must equal a full K3 pass. A failed
witness exits non-zero.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def witness_check(km, rt):
    """One more (untimed) iteration, checked against brute force and a full K3 pass."""
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
        from dalgo.parallel import comm         # the full path keeps only the global sums
        comm.all_reduce_sum(S_ref)
        comm.all_reduce_sum(c_ref)
        S_m, c_m = km.S.double(), km.cnt
    err = float(((S_ref.double() - S_m.double()).abs().max() /
                 (1.0 + S_ref.double().abs().max())).item())
    counts_equal = bool(torch.equal(c_ref, c_m))
    return {"iteration": km.t, "path": "bounds" if km.bounds else (
                "incremental" if km.incremental else "full"),
            "assignment_agreement_vs_brute_force": agree, "disagreements": int(diff.numel()),
            "max_disagreement_gap": max_gap, "distance_slack": slack,
            "counts_equal": counts_equal, "sums_max_rel_err": err,
            "passed": bool(agree > 0.999 and max_gap <= slack and counts_equal and err < 1e-4)}


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5, help="Lloyd iterations of the job "
                    "(the reference's n_iterations, k-means.py:18)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="ranks (one per GPU); started here as a torchrun child when > 1")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"])
    ap.add_argument("--no-witness", action="store_true")
    ap.add_argument("--no-candidates", action="store_true",
                    help="filtered iterations without the candidate-pruned K2 tiles")
    ap.add_argument("--no-bound-filter", action="store_true",
                    help="plain (full K2 every iteration) Lloyd with the incremental K3")
    ap.add_argument("--deadline-s", type=float, default=420.0)
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    from dalgo.parallel.launch import check_world, self_launch
    rc = self_launch(a.gpus, __file__, argv, device=a.device, backend=a.backend, tag="kmeans_bench")
    if rc is not None:
        sys.exit(rc)
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.parallel import comm, runtime
    from dalgo.parallel.sharding import even_slices
    runtime.arm_watchdog(a.deadline_s, tag="kmeans_bench")
    rt = runtime.init(backend=a.backend, device=a.device, app_name="kmeans-bench", timeout_s=120)
    W = rt.world_size
    check_world(a.gpus, W, "kmeans_bench")
    lo, hi = even_slices(a.rows, W)[rt.rank]
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    cuda = rt.device.type == "cuda"

    # process warm-up (separate, small model; discarded)
    wn = min(1_000_000, a.rows)
    wlo, whi = even_slices(wn, W)[rt.rank]
    Xw = blobs(wn, a.dim, a.k, row_range=(wlo, whi), device=rt.device, dtype=dtype, seed=3)
    kw = KMeans(KMeansConfig(k=min(a.k, wn), n_iterations=2, seed=5), Xw, wlo, wn)
    kw.step()
    kw.step()
    del kw, Xw

    t0 = time.time()
    X = blobs(a.rows, a.dim, a.k, row_range=(lo, hi), device=rt.device, dtype=dtype, seed=7)
    rt.synchronize()
    gen = time.time() - t0

    def ev():
        if not cuda:
            return time.perf_counter()
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def span(e0, e1):
        return (e1 - e0) * 1e3 if not cuda else e0.elapsed_time(e1)

    rt.barrier()
    rt.synchronize()
    t = time.perf_counter()
    marks = [ev()]
    km = KMeans(KMeansConfig(k=a.k, n_iterations=a.iters, seed=1,
                             bound_filter=not a.no_bound_filter,
                             candidates=not a.no_candidates), X, lo, a.rows)
    marks.append(ev())
    for _ in range(a.iters):
        km.step()
        marks.append(ev())
    rt.synchronize()
    rt.barrier()
    rt.synchronize()
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=rt.device)
    comm.all_reduce_max(el)
    job_ms = float(el.item()) * 1e3
    init_ms = span(marks[0], marks[1])
    iter_ms = [span(marks[i], marks[i + 1]) for i in range(1, len(marks) - 1)]
    sse_last = km.sse.clone()
    comm.all_reduce_sum(sse_last)
    active = km.active_history
    moved = km.changed_history
    witness = None if a.no_witness else witness_check(km, rt)
    flops = 2.0 * a.rows * a.k * a.dim
    if rt.is_main:
        steady = iter_ms[1:]
        print(json.dumps({
            "metric": "k-means points/sec (whole node)",
            "measured": f"reference job: init + {a.iters} Lloyd iterations, iteration 1 included",
            "value": a.rows * a.iters / (job_ms / 1e3), "unit": "points/s", "n_gpus": W,
            "job_ms": job_ms, "ms_per_iter": job_ms / a.iters, "iterations": a.iters,
            "init_ms_rank0": init_ms, "iteration_ms_rank0": iter_ms,
            "first_iteration_ms_rank0": iter_ms[0] if iter_ms else None,
            "steady_ms_per_iter_rank0": sum(steady) / len(steady) if steady else None,
            "full_pass_tflops_per_gpu": (flops / W / (iter_ms[0] / 1e3) / 1e12) if iter_ms else None,
            "reassigned_rows_per_iter_rank0": active, "moved_rows_per_iter_rank0": moved,
            "bound_filter": km.bounds, "candidate_pruning": getattr(km, "_cand", None) is not None,
            "incremental_k3": km.incremental,
            "sse_last_iteration": float(sse_last.item()),
            "correctness_witness": witness,
            "config": {"rows": a.rows, "dim": a.dim, "k": a.k, "dtype": a.dtype,
                       "init": "takeSample-style: k distinct seeded rows (k-means.py:53)"},
            "timing": "model construction + iterations 1..%d inside the clock (MAX over ranks); "
                      "process warmed up on a separate 1M-row model" % a.iters,
            "datagen_s": gen}), flush=True)
    runtime.shutdown()
    runtime.arm_watchdog(0)
    if witness is not None and not witness["passed"]:
        raise SystemExit(f"[kmeans_bench] correctness witness failed: {witness}")


if __name__ == "__main__":
    main()
