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

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    ap.add_argument("--noise", type=float, default=1.0,
                    help="blob noise (1 = well separated; 4 = overlapping clusters, the hard case "
                         "for the bound filters)")
    ap.add_argument("--dense", default="auto", choices=["auto", "always", "never", "device"],
                    help="filtered iterations on the dense top-2 K2 (auto: right after the full pass)")
    ap.add_argument("--no-drift", action="store_true",
                    help="candidate lists without the centre-shift pruning")
    ap.add_argument("--deadline-s", type=float, default=420.0)
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    from dalgo.parallel.launch import check_world, self_launch
    rc = self_launch(a.gpus, __file__, argv, device=a.device, backend=a.backend, tag="kmeans_bench")
    if rc is not None:
        sys.exit(rc)
    from dalgo.apps.jobs import kmeans_job
    from dalgo.parallel import runtime
    runtime.arm_watchdog(a.deadline_s, tag="kmeans_bench")
    rt = runtime.init(backend=a.backend, device=a.device, app_name="kmeans-bench", timeout_s=120)
    check_world(a.gpus, rt.world_size, "kmeans_bench")
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    out = kmeans_job(rt, a.rows, a.dim, a.k, a.iters, dtype=dtype, noise=a.noise,
                     bound_filter=not a.no_bound_filter, candidates=not a.no_candidates,
                     witness=not a.no_witness, dense=a.dense, drift=not a.no_drift)
    if rt.is_main:
        print(json.dumps(out), flush=True)
    runtime.shutdown()
    runtime.arm_watchdog(0)
    w = out["correctness_witness"]
    if w is not None and not w["passed"]:
        raise SystemExit(f"[kmeans_bench] correctness witness failed: {w}")


if __name__ == "__main__":
    main()
