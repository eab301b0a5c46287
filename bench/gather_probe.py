#!/usr/bin/env python3
"""Ceiling probes for K1's access shape (sorted Bernoulli(frac) list of 2-KB bf16 rows):
register gathers (default / nt policy) vs LDS-DMA gathers into a per-wave ring (depth 4 /
6 / 8 rows, default / nt). Interleaved rounds in one process; best and median GB/s."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalgo.ops import _ext  # noqa: E402
from dalgo.ops import random as R  # noqa: E402

MODES = {0: "reg", 1: "reg-nt", 2: "lds4", 3: "lds4-nt", 4: "lds6", 5: "lds6-nt", 6: "lds8", 7: "lds8-nt"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--frac", type=float, default=0.1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--arms", default="0:2048,1:2048,2:256,2:512,3:256,3:512,4:256,5:256,6:256,7:256")
    a = ap.parse_args()
    assert _ext.load()
    dev = torch.device("cuda", 0)
    X = torch.empty((a.rows, 1024), dtype=torch.bfloat16, device=dev)
    R.philox_fill_(X, D=1024, seed=1, stream=1, a=-1, b=1)
    sel = torch.nonzero(torch.rand(a.rows, device=dev) < a.frac).flatten().to(torch.int32)
    arms = [tuple(int(x) for x in s.split(":")) for s in a.arms.split(",")]
    ref = None
    for m, g in arms:   # every form must fold the same rows to the same word
        o = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.ops.dalgo.hbm_gather_rows(X, sel, o, g | (m << 20))
        torch.cuda.synchronize()
        print(json.dumps({"mode": MODES[m], "grid": g, "check": int(o.item())}))
    res = {arm: [] for arm in arms}
    o = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(a.rounds):
        for m, g in arms:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                torch.ops.dalgo.hbm_gather_rows(X, sel, o, g | (m << 20))
            torch.cuda.synchronize()
            res[(m, g)].append((time.perf_counter() - t0) / 10)
    nbytes = sel.numel() * 2048
    for (m, g), ts in sorted(res.items(), key=lambda kv: min(kv[1])):
        ts.sort()
        print(json.dumps({"mode": MODES[m], "grid": g, "us_best": ts[0] * 1e6,
                          "GBps_best": nbytes / ts[0] / 1e9, "GBps_median": nbytes / ts[len(ts) // 2] / 1e9}))


if __name__ == "__main__":
    main()
