"""Run-length census and timing of the split key sort (graph_build.hip gb_sort over the bits
above the source offset + gb_run_sort) on the scale-26 PageRank keys: builds the graph
with keep_keys, prints the histogram of run lengths (runs = keys equal above the
low bits left to the run sort) and times, on a random permutation of the same keys, the full 52-bit
sort, the 39-bit sort and the run sort (CUDA events, after a warm call each)."""
import argparse
import json
import os
import sys

import torch

sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.apps.pagerank_app import build_rmat_native, rmat_input   # noqa: E402
from dalgo.ops import _ext                                           # noqa: E402
from dalgo.ops import graph as G                                     # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=26)
ap.add_argument("--no-census", action="store_true", help="skip the run-length histogram")
ap.add_argument("--lo-bits", type=int, default=None, help="split point (default: build_native's)")
a = ap.parse_args()
dev = torch.device("cuda")
edges, _ = rmat_input(a.scale, 16, dev, seed=1)
ng = build_rmat_native(edges, a.scale, 0, 1, dev, keep_keys=True)
del edges
K = ng.keys[: ng.n_keys] if hasattr(ng, "n_keys") else ng.keys
n = K.numel()
nbits = ng.key_shift + max(1, (int(ng.blk_base.numel()) - 1).bit_length())   # as build_native
lo_bits = G.sort_split_bits(nbits) if a.lo_bits is None else a.lo_bits
if not a.no_census:
    hi = K >> lo_bits
    _, cnt = torch.unique_consecutive(hi, return_counts=True)
    del hi
    edges_b = [1, 2, 4, 8, 16, 64, 256, 1024, 8192, 1 << 40]
    hist = {}
    lo = 0
    for e in edges_b:
        m = (cnt > lo) & (cnt <= e)
        hist[f"{lo + 1}-{e}"] = {"runs": int(m.sum()), "keys": int(cnt[m].sum())}
        lo = e
    print(json.dumps({"n_keys": n, "nbits": nbits, "lo_bits": lo_bits, "runs": int(cnt.numel()),
                      "max_run": int(cnt.max()), "hist": hist}))
    del cnt
ops = _ext.ops()
perm = K[torch.randperm(n, device=dev)]
out = torch.empty_like(perm)


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return min(ts)


t_full = timed(lambda: ops.gb_sort(perm, n, nbits, out, 0))
t_hi = timed(lambda: ops.gb_sort(perm, n, nbits, out, lo_bits))
work = out.clone()


counts = []


def run_sort():
    work.copy_(out)
    counts.append(ops.gb_run_sort(work, n, lo_bits))


t_copy = timed(lambda: work.copy_(out))
t_run = timed(run_sort) - t_copy
ok = torch.equal(work, K)
print(json.dumps({"sort_full_ms": t_full, "sort_hi_ms": t_hi, "run_sort_ms": t_run, "copy_ms": t_copy,
                  "equal": bool(ok),
                  "long_runs": counts[-1].tolist()}))
