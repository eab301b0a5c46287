#!/usr/bin/env python3
"""K5 ALS row solve: (R F) Ginv over an m x n f32 R (default 100k x 50k, k = 64).

Times every DALGO_ALS_VARIANT of the hand-written MFMA kernel (csrc/kernels/als.hip)
against the library GEMM form torch.matmul(torch.matmul(R, F), Ginv), interleaved
over rounds (best of R), and reports the effective R stream rate. Then times one full
ALS sweep (both half-sweeps) of dalgo.models.als on the same shape."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="100000,50000,64")
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sweep", action="store_true", help="also time a full ALS sweep")
    a = ap.parse_args()
    from dalgo.models.als import rows_solve
    from dalgo.ops import random as drandom
    dev = torch.device("cuda", 0)
    m, n, k = (int(x) for x in a.shape.split(","))
    R = torch.empty(m, n, device=dev)
    drandom.philox_fill_(R, D=n, seed=1, stream=1, a=0.0, b=16.0)
    F = torch.rand(n, k, device=dev) - 0.3
    Gi = torch.rand(k, k, device=dev) - 0.5
    gb = m * n * 4 / 1e9
    best = {}
    for _ in range(a.rounds):
        for v in a.variants.split(","):
            os.environ["DALGO_ALS_VARIANT"] = v
            dt = timed(lambda: rows_solve(R, F, Gi), a.reps)
            best[f"v{v}"] = min(best.get(f"v{v}", 1e9), dt)
        dt = timed(lambda: (R @ F) @ Gi, a.reps)
        best["torch"] = min(best.get("torch", 1e9), dt)
    os.environ.pop("DALGO_ALS_VARIANT", None)
    ref = ((R[:2048].double() @ F.double()) @ Gi.double())
    err = ((rows_solve(R, F, Gi)[:2048].double() - ref).abs().max() / ref.abs().max()).item()
    out = {"shape": [m, n, k], "max_rel_err_first_2048_rows": err,
           "ms": {key: v * 1e3 for key, v in best.items()},
           "R_stream_TBps": {key: gb / v / 1e3 for key, v in best.items()}}
    if a.sweep:
        from dalgo.models.als import ALS, ALSConfig
        del R
        torch.cuda.empty_cache()
        als = ALS(ALSConfig(m=m, n=n, k=k, seed=1), device=dev)
        dt = timed(als.step, 3)
        out["als_sweep_ms"] = dt * 1e3
        out["rmse"] = als.rmse()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
