#!/usr/bin/env python3
"""Per-rank compute of the BASELINE workloads at W = 1, 2, 4, 8, measured on ONE MI355X.

The driver measures the real N-GPU scaling of bench.py on an 8-GPU node; this script
measures what each rank computes per step at every W (the rank's share of the global
problem, on real hardware) and reports the communication each step adds, so the
scaling curve can be read as (per-rank compute) + (collective):

  ssgd     K1 + K8 per step on rows/W of the 10M x 1024 bf16 set    + one 4 KB all-reduce
  kmeans   assign + accumulate + update on 100M/W points (k = 1024)  + [k x 128 f32 + k] all-reduce
  pagerank rank 0's destination slice of the R-MAT scale-26 graph (dealt relabeling,
           ghost-relabeled edge list): SpMV + update (K4b and pull)  + ghost all_to_all (floats)

No collective runs here (one process); the compute-only throughput W x share / time is an
upper bound that the measured SCALE run is compared against.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def ssgd(worlds, rows=10_000_000, dim=1024):
    from dalgo.data.datasets import synthetic_logistic
    from dalgo.models.localsgd import ParallelSGD, SGDConfig
    from dalgo.parallel import runtime
    from dalgo.parallel.sharding import make_layout
    rt = runtime.get()
    out = {}
    for W in worlds:
        n = rows // W
        lay = make_layout(n, 1, 1, 0, spark_compatible=False)
        d = synthetic_logistic(n, dim, device=rt.device, dtype=torch.bfloat16)
        m = ParallelSGD(SGDConfig(algo="ssgd", n_workers=1, eval_every=0), d, lay, rt)
        dt = timed(m.step, 100 if W > 1 else 30)
        per_rank = 0.1 * n / dt
        out[f"W{W}"] = {"rows_per_rank": n, "step_us": dt * 1e6,
                        "compute_only_samples_per_s_whole_job": per_rank * W,
                        "allreduce_bytes_per_step": 4 * (dim + 2)}
        del d, m
        torch.cuda.empty_cache()
    return out


def kmeans(worlds, rows=100_000_000, dim=128, k=1024):
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    out = {}
    for W in worlds:
        n = rows // W
        X = blobs(n, dim, k, device="cuda", dtype=torch.bfloat16, seed=7)
        km = KMeans(KMeansConfig(k=k, seed=1), X, 0, n)
        dt = timed(km.step, 3, warm=1)
        out[f"W{W}"] = {"points_per_rank": n, "iter_ms": dt * 1e3,
                        "compute_only_points_per_s_whole_job": rows / dt,
                        "allreduce_bytes_per_iter": 4 * k * km.DP + 8 * k}
        del X, km
        torch.cuda.empty_cache()
    return out


def pagerank(worlds, scale=26, edge_factor=16):
    from dalgo.apps.pagerank_app import deal_ids
    from dalgo.ops import graph as G
    dev = torch.device("cuda", 0)
    n = 1 << scale
    E = edge_factor * n
    chunk = 1 << 26
    deg = torch.zeros(n, dtype=torch.int64, device=dev)
    for off in range(0, E, chunk):
        s, _ = G.rmat_edges(min(chunk, E - off), scale, seed=2, e_off=off, device=dev)
        deg += torch.bincount(s.long(), minlength=n)
    order = torch.argsort(-deg * n - torch.arange(n, device=dev, dtype=torch.int64))
    out = {}
    for W in worlds:
        nid = deal_ids(order, n, W)
        sl = G.vertex_slices(n, W)
        parts = []
        for off in range(0, E, chunk):
            s, d = G.rmat_edges(min(chunk, E - off), scale, seed=2, e_off=off, device=dev)
            s, d = nid[s.long()], nid[d.long()]
            keep = d < sl                                          # rank 0's slice
            parts.append((s[keep].to(torch.int32), (d[keep]).to(torch.int32)))
        sh = G.merge_shards(parts, 0, sl, n, sl)
        del parts
        Ei = sh.n_edges
        src = sh.src[:Ei].long()
        remote = src >= sl
        ghosts = torch.unique(src[remote])
        loc = torch.where(remote, sl + torch.searchsorted(ghosts, src), src)
        src_local = torch.full_like(sh.src, -1)
        src_local[:Ei] = loc.to(torch.int32)
        g = G.GraphShard(src_local, sh.dstl, Ei, 0, sl, n, sl)
        c = torch.rand(sl + ghosts.numel(), device=dev) * 1e-8
        acc = torch.zeros(sl, device=dev)
        pres = torch.zeros(sl, dtype=torch.int32, device=dev)
        od = torch.randint(1, 20, (sl,), dtype=torch.int32, device=dev)
        r = torch.zeros(sl, device=dev)

        def it():
            acc.zero_()
            pres.zero_()
            G.pr_spmv(g, c, acc, pres)
            G.pr_update(acc, pres, od, 0.15, 1.0 / n, 0, r, c[:sl])
        dt = timed(it, 5)
        # the overlapped ghost exchange's form: own-slice sources first (no exchange
        # needed), then the ghost sources adding into the same rows
        own = loc < sl

        def part(m):
            k = int(m.sum().item())
            kp = (k + 3) // 4 * 4
            s_ = torch.full((kp,), -1, dtype=torch.int32, device=dev)
            d_ = torch.full((kp,), -1, dtype=torch.int32, device=dev)
            s_[:k] = loc[m].to(torch.int32)
            d_[:k] = sh.dstl[:Ei][m]
            return G.GraphShard(s_, d_, k, 0, sl, n, sl)
        g_own, g_gh = part(own), part(~own)

        def it_split():
            acc.zero_()
            pres.zero_()
            G.pr_spmv(g_own, c, acc, pres)
            G.pr_spmv(g_gh, c, acc, pres, accumulate=True)
            G.pr_update(acc, pres, od, 0.15, 1.0 / n, 0, r, c[:sl])
        dt_split = timed(it_split, 5) if W > 1 else dt
        del g_own, g_gh
        # K4b (default SpMV) over the same ghost-relabeled edge list, update fused
        lay = G.build_blocked(g)
        upd = dict(outdeg=od, q=0.15, invN=1.0 / n, mode=0, r=r, c=c[:sl])

        def it_pb():
            G.pb_spmv(lay, c, acc, pres, update=upd)
        dt_pb = timed(it_pb, 5)
        del lay
        out[f"W{W}"] = {"edges_rank0": Ei, "iter_ms_rank0_k4b": dt_pb * 1e3,
                        "compute_only_edges_per_s_whole_job_k4b": E / dt_pb,
                        "iter_ms_rank0": dt * 1e3,
                        "iter_ms_rank0_split": dt_split * 1e3,
                        "ghost_edge_share_rank0": float((~own).float().mean().item()),
                        "compute_only_edges_per_s_whole_job": E / dt,
                        "ghost_floats_rank0": int(ghosts.numel()),
                        "allgather_floats_per_rank": (W - 1) * sl}
        del sh, g, c, src, loc, src_local
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--only", default="ssgd,kmeans,pagerank")
    a = ap.parse_args()
    from dalgo.parallel import runtime
    runtime.init(device="cuda")
    worlds = [int(x) for x in a.worlds.split(",")]
    res = {}
    for name in a.only.split(","):
        res[name] = {"ssgd": ssgd, "kmeans": kmeans, "pagerank": pagerank}[name](worlds)
        print(json.dumps({name: res[name]}), flush=True)
    runtime.shutdown()


if __name__ == "__main__":
    main()
