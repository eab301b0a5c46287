#!/usr/bin/env python3
"""SSGD-shaped K1 launches: balanced slices (K7 selection one step ahead on a side
stream, K1 LIST build) vs the in-register Bernoulli walk over static row ranges.

Times back-to-back gradient launches (HIP events, both forms in the same process,
alternating) and checks that both forms draw the same minibatch each step.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1250000,10000000")
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--frac", type=float, default=0.1)
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    from dalgo.ops import lr as L
    from dalgo.ops import random as R
    dev = torch.device("cuda", 0)
    for n in [int(v) for v in a.rows.split(",")]:
        X = torch.empty((n, a.dim), dtype=torch.bfloat16, device=dev)
        R.philox_fill_(X, seed=3)
        y = (torch.rand(n, device=dev) < 0.5).float()
        W = torch.randn((1, a.dim + 1), device=dev) * 0.01
        seg = torch.tensor([0, n], dtype=torch.int64, device=dev)
        G = torch.zeros((1, a.dim + 1), device=dev)
        C = torch.zeros(1, device=dev)

        def run(bal, s):
            L.LR_BALANCED = bal
            L.lr_grad(X, y, W, seg, D=a.dim, frac=a.frac, seed=42, step=s, G=G, C=C)

        same = True
        for s in range(4):
            run(False, s)
            c0, g0 = C.clone(), G.clone()
            run(True, s)
            torch.cuda.synchronize()
            same = same and torch.equal(c0, C) and bool(torch.allclose(g0, G, rtol=1e-3, atol=1e-2))
        res = {"same_minibatch": same}
        for bal in (False, True, False, True):
            for s in range(5):
                run(bal, 1000 + s)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in range(a.steps):
                run(bal, 2000 + s)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault("list_us" if bal else "walk_us", []).append(
                round(e0.elapsed_time(e1) / a.steps * 1e3, 2))
        print(json.dumps({"rows": n, **res}), flush=True)
        del X
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
