#!/usr/bin/env python3
"""A/B sweep of the fused sampled-gradient kernel (K1+K7) launch shapes.

Interleaved rounds in ONE process (guide §5.4 rule 24): every (variant, blocks)
arm runs once per round, R rounds, median/min reported as effective GB/s of
sampled rows (rows * D * 2 B) — the HBM-gather roofline is ~5.7-6.3 TB/s.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalgo.ops import lr as L  # noqa: E402
from dalgo.ops import random as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--frac", type=float, default=0.1)
    ap.add_argument("--ref", action="store_true", help="also time a plain HBM read of X (torch sum) and a D2D copy")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--blocks", default="256,512,768,1024,2048")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X = torch.empty((a.rows, a.dim), dtype=torch.bfloat16, device=dev)
    R.philox_fill_(X, D=a.dim, seed=1, stream=1, a=-1, b=1)
    y = (torch.rand(a.rows, device=dev) < 0.5).float()
    W = torch.randn(1, a.dim + 1, device=dev) * 0.05
    seg = torch.tensor([0, a.rows], dtype=torch.int64, device=dev)
    G = torch.zeros(1, a.dim + 1, device=dev)
    C = torch.zeros(1, device=dev)
    arms = [(int(v), int(b)) for v in a.variants.split(",") for b in a.blocks.split(",")]
    res = {arm: [] for arm in arms}
    step = 0
    for arm in arms:  # warm + correctness: all arms must agree bitwise on C, closely on G
        L.lr_grad(X, y, W, seg, D=a.dim, frac=a.frac, step=0, G=G, C=C, variant=arm[0], target_blocks=arm[1])
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for arm in arms:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                step += 1
                L.lr_grad(X, y, W, seg, D=a.dim, frac=a.frac, step=step, G=G, C=C,
                          variant=arm[0], target_blocks=arm[1], g_is_zero=True)
            torch.cuda.synchronize()
            res[arm].append((time.perf_counter() - t0) / a.reps)
    rows = a.rows * a.frac
    if a.ref:
        nbytes = X.numel() * 2
        Xf = X.view(torch.int32)
        buf = torch.empty_like(X)
        for name, fn in [("copy", lambda: buf.copy_(X)), ("sum_i32", lambda: Xf.sum(dtype=torch.int64))]:
            fn(); torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 5
            mult = 2 if name == "copy" else 1
            print(json.dumps({"ref": name, "GBps": nbytes * mult / dt / 1e9, "ms": dt * 1e3}))
        del buf
        for grid in (256, 512, 1024, 2048, 4096, 8192):
            for unroll in (8, -4, -8):
                o = torch.zeros(grid, dtype=torch.int32, device=dev)
                torch.ops.dalgo.hbm_read(X, o, unroll); torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    torch.ops.dalgo.hbm_read(X, o, unroll)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / 5
                print(json.dumps({"ref": f"hbm_read grid={grid} unroll={unroll}", "GBps": nbytes / dt / 1e9}))
    if a.ref:
        # the minibatch access shape itself: the same Bernoulli(frac) rows, sorted
        from dalgo.utils import philox  # noqa: F401  (documents the sampling stream)
        n = X.shape[0]
        sel = torch.nonzero(torch.rand(n, device=dev) < a.frac).flatten().to(torch.int32)
        o = torch.zeros(1, dtype=torch.int32, device=dev)
        for grid in (512, 1024, 2048, 4096, 8192):
            torch.ops.dalgo.hbm_gather_rows(X, sel, o, grid); torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                torch.ops.dalgo.hbm_gather_rows(X, sel, o, grid)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            print(json.dumps({"ref": f"gather_rows grid={grid}", "rows": int(sel.numel()),
                              "GBps": sel.numel() * X.stride(0) * 2 / dt / 1e9, "us": dt * 1e6}))
    out = []
    for arm, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        out.append({"variant": arm[0], "blocks": arm[1], "us_median": med * 1e6, "us_min": ts[0] * 1e6,
                    "GBps_median": rows * a.dim * 2 / med / 1e9, "Gsamples_s": rows / med / 1e9})
    out.sort(key=lambda d: d["us_median"])
    for d in out:
        print(json.dumps(d))


if __name__ == "__main__":
    main()
