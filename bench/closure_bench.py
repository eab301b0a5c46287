#!/usr/bin/env python3
"""K9 sparse transitive-closure bench: random sparse digraph, hash-set frontier engine.

Reference: graph_computation/transitive_closure.py:31-40 (join + union + distinct +
count per round). The graph has n vertices and avg_deg * n uniform random edges;
avg_deg < 1 keeps the closure sparse (no giant strongly connected component).
Reports rounds, |closure|, candidates examined, time per round and candidates/s
(each candidate = one join output row that goes through dedup + merge). Pass
--torch-ref to time the torch (repeat_interleave / unique / isin / sort) engine on
the same graph for comparison.

Run: python bench/closure_bench.py [--n 1048576 --avg-deg 0.9]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--avg-deg", type=float, default=0.9)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--torch-ref", action="store_true")
    a = ap.parse_args()
    from dalgo.models.transitive_closure import SparseClosure
    from dalgo.parallel import runtime
    rt = runtime.init(device="cuda")
    g = torch.Generator().manual_seed(a.seed)
    e = int(a.avg_deg * a.n)
    src = torch.randint(0, a.n, (e,), generator=g)
    dst = torch.randint(0, a.n, (e,), generator=g)
    out = {"n": a.n, "edges": e}
    engines = [("hash-set K9", False)] + ([("torch sort/unique/isin", True)] if a.torch_ref else [])
    for name, ref in engines:
        tc = SparseClosure(src, dst, n=a.n, device=rt.device)
        if ref:
            P = tc.paths()
            tc.gpu = False                 # same object, torch engine on the GPU tensors
            tc.P = P
            tc.delta = P
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = tc.run()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rec = {"engine": name, "rounds": len(res.counts) - 1, "paths": res.n_paths,
               "seconds": el, "ms_per_round": el / max(1, len(res.counts) - 1) * 1e3}
        if not ref:
            cand = sum(tc.rounds_candidates)
            rec.update(candidates=cand, candidates_per_s=cand / el,
                       table_slots=tc.table.numel())
        out[name] = rec
        print(json.dumps(rec), flush=True)
    runtime.shutdown()


if __name__ == "__main__":
    main()
