#!/usr/bin/env python3
"""PageRank benchmark (BASELINE config #5: synthetic 1B-edge power-law graph).

Graph500 R-MAT (a,b,c = 0.57,0.19,0.19), scale 26, edge factor 16 = 1.07B edges,
vertex ids scrambled. Headline = the reference's JOB (graph_computation/pagerank.py:
41-57): adjacency build from the generated edge list (degree relabeling, dedup, out-
degrees, K4b layout) + 10 iterations, ``job_ms``; the per-iteration SpMV rate (edges/s)
is secondary. Destination-partitioned over the ranks. A correctness witness runs after
the timed region: one more K4b step against the pull K4 SpMV from the same state; the
ranks must agree to f32 rounding, else the bench exits non-zero (dalgo.apps.jobs).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10, help="iterations of the job "
                    "(graph_computation/pagerank.py:18)")
    ap.add_argument("--steps", type=int, default=10, help="iterations timed alone after the job")
    ap.add_argument("--semantics", default="reference")
    ap.add_argument("--no-reorder", action="store_true", help="keep scrambled R-MAT vertex ids")
    ap.add_argument("--spmv", default="blocked", choices=["pull", "blocked"])
    ap.add_argument("--no-witness", action="store_true")
    ap.add_argument("--deadline-s", type=float, default=420.0)
    ap.add_argument("--pool-gb", type=float, default=96.0,
                    help="device memory held by the caching allocator before the clock")
    ap.add_argument("--no-warm", action="store_true",
                    help="skip the scale-16 process warm-up before the clock")
    ap.add_argument("--bin-width", type=int, default=16384)
    ap.add_argument("--chunk", type=int, default=1 << 40)
    ap.add_argument("--tile", type=int, default=16384)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="ranks (one per GPU); started here as a torchrun child when > 1")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"])
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    from dalgo.parallel.launch import check_world, self_launch
    rc = self_launch(a.gpus, __file__, argv, device=a.device, backend=a.backend, tag="pagerank_bench")
    if rc is not None:
        sys.exit(rc)
    from dalgo.apps.jobs import pagerank_job
    from dalgo.parallel import runtime
    runtime.arm_watchdog(a.deadline_s, tag="pagerank_bench")
    rt = runtime.init(backend=a.backend, device=a.device, app_name="pagerank-bench", timeout_s=120)
    check_world(a.gpus, rt.world_size, "pagerank_bench")
    out = pagerank_job(rt, a.scale, a.edge_factor, a.iters, spmv=a.spmv, semantics=a.semantics,
                       witness=not a.no_witness, reorder=not a.no_reorder, bin_width=a.bin_width,
                       chunk=a.chunk, tile=a.tile, timed_iters=a.steps, pool_gb=a.pool_gb,
                       warm=not a.no_warm)
    if rt.is_main:
        print(json.dumps(out), flush=True)
    runtime.shutdown()
    runtime.arm_watchdog(0)
    w = out["correctness_witness"]
    if w is not None and not w["passed"]:
        raise SystemExit(f"[pagerank_bench] correctness witness failed: {w}")


if __name__ == "__main__":
    main()
