#!/usr/bin/env python3
"""PageRank benchmark (BASELINE config: synthetic 1B-edge power-law graph).

Graph500 R-MAT (a,b,c = 0.57,0.19,0.19), scale 26, edge factor 16 = 1.07B edges,
vertex ids scrambled, deduplicated (distinct()). Destination-partitioned over the
ranks. Reports edges/s (whole job, edges per iteration / iteration time). The phase
split comes from HIP events on one warm-up step. A correctness witness runs after the
timed region (untimed): one iteration of the benchmarked SpMV (K4b by default: fixed-point
blocked, update fused) against the pull K4 SpMV from the same state; the ranks must agree
to f32 rounding, else the bench exits non-zero.
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
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--semantics", default="reference")
    ap.add_argument("--no-reorder", action="store_true", help="keep scrambled R-MAT vertex ids")
    ap.add_argument("--spmv", default="blocked", choices=["pull", "blocked"])
    ap.add_argument("--no-witness", action="store_true")
    ap.add_argument("--deadline-s", type=float, default=420.0)
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
    from dalgo.apps.pagerank_app import rmat_shard
    from dalgo.models.pagerank import PageRank, PageRankConfig
    from dalgo.ops import graph as G
    from dalgo.parallel import comm, runtime
    runtime.arm_watchdog(a.deadline_s, tag="pagerank_bench")
    rt = runtime.init(backend=a.backend, device=a.device, app_name="pagerank-bench", timeout_s=120)
    W = rt.world_size
    check_world(a.gpus, W, "pagerank_bench")
    t0 = time.time()
    shard, n_gen = rmat_shard(a.scale, a.edge_factor, rt.rank, W, rt.device, reorder=not a.no_reorder)
    rt.synchronize()
    build_s = time.time() - t0
    E = comm.all_reduce_count(shard.n_edges, device=rt.device)
    pr = PageRank(PageRankConfig(semantics=a.semantics, spmv=a.spmv, bin_width=a.bin_width,
                                 chunk=a.chunk, tile=a.tile), shard, W)
    from dalgo.utils.obs import PhaseTimer
    phases = {}
    for i in range(max(a.warmup, 1)):
        if i == 0:
            pr.timer = PhaseTimer(rt.device)   # HIP events inside step(): the phase split
        pr.step()
        if i == 0:
            rt.synchronize()
            phases = pr.timer.summary()
            pr.timer = None
    rt.synchronize()
    done = pr.t
    xf = torch.tensor([pr.exchange_floats()], dtype=torch.int64, device=rt.device)
    comm.all_reduce_sum(xf)
    rt.barrier(); rt.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        pr.step()
    rt.synchronize(); rt.barrier(); rt.synchronize()
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=rt.device)
    comm.all_reduce_max(el)
    ms = float(el.item()) / a.steps * 1e3
    witness = None
    if not a.no_witness:
        # one more iteration of the benchmarked SpMV vs the pull SpMV from the same state
        ref = PageRank(PageRankConfig(semantics=a.semantics, spmv="pull", exchange=pr.exchange),
                       shard, W)
        ref.load_state_dict(pr.state_dict())
        pr.step()
        ref.step()
        rt.synchronize()
        r1, r0 = pr.r.double(), ref.r.double()
        both = (r1 >= 0) & (r0 >= 0)
        err = torch.tensor([float(((r1 - r0).abs() * both).max().item()),
                            float((r1 >= 0).ne(r0 >= 0).sum().item())], dtype=torch.float64,
                           device=rt.device)
        comm.all_reduce_max(err)
        scale = torch.tensor([float(r0.abs().max().item())], dtype=torch.float64, device=rt.device)
        comm.all_reduce_max(scale)
        rel = float(err[0].item()) / max(float(scale.item()), 1e-30)
        witness = {"vs": "pull K4 SpMV, same state", "max_rel_err": rel,
                   "presence_mismatches": int(err[1].item()), "iteration": pr.t,
                   "passed": bool(rel < 1e-5 and int(err[1].item()) == 0)}
    if rt.is_main:
        print(json.dumps({
            "metric": "PageRank edges/sec (whole node)", "value": E / (ms / 1e3), "unit": "edges/s",
            "n_gpus": W, "ms_per_iter": ms, "edges_dedup": E, "edges_generated": n_gen,
            "vertices": 1 << a.scale, "degree_reordered": not a.no_reorder, "spmv": pr.spmv, "phases_ms_rank0": phases, "graph_build_s": build_s,
            "timed_steps": a.steps, "steps_before_timing": done, "correctness_witness": witness,
            "exchange": pr.exchange, "exchange_MB_per_iter_all_ranks": int(xf.item()) * 4 / 1e6,
            "blocked_layout_rank0": None if pr.layout is None else {
                "chunks": pr.layout.n_chunks, "entries": pr.layout.n_entries,
                "entries_per_edge": pr.layout.n_entries / max(shard.n_edges, 1),
                "work_items": int(pr.layout.wi_bin.numel()), "split_bins": int(pr.layout.split_bin.numel()),
                "bin_width": pr.layout.bin_width},
            "allgather_MB_per_iter_all_ranks": (W - 1) * W * shard.slice_size * 4 / 1e6}), flush=True)
    runtime.shutdown()
    runtime.arm_watchdog(0)
    if witness is not None and not witness["passed"]:
        raise SystemExit(f"[pagerank_bench] correctness witness failed: {witness}")


if __name__ == "__main__":
    main()
