#!/usr/bin/env python3
"""Throughput of the smaller workloads: Monte-Carlo pi (K6), transitive closure
(K9 dense boolean MFMA GEMM), ALS half-sweeps (Gram + K5 inverse + GEMMs)."""
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
    ap.add_argument("--mc-samples", type=int, default=10_000_000_000)
    ap.add_argument("--tc-n", type=int, default=16384)
    ap.add_argument("--als", default="100000,50000,64")
    a = ap.parse_args()
    from dalgo.models.als import ALS, ALSConfig
    from dalgo.models.transitive_closure import DenseClosure
    from dalgo.ops import _ext
    from dalgo.ops import random as R
    dev = torch.device("cuda", 0)
    out = {}
    # Monte Carlo
    dt = timed(lambda: R.mc_pi_count(a.mc_samples, seed=1, device=dev), 3)
    cnt = int(R.mc_pi_count(a.mc_samples, seed=1, device=dev).item())
    out["monte_carlo"] = {"samples": a.mc_samples, "s": dt, "samples_per_s": a.mc_samples / dt,
                          "pi": 4.0 * cnt / a.mc_samples}
    # transitive closure step (dense, n x n)
    n = a.tc_n
    g = torch.Generator(device=dev).manual_seed(0)
    e = 4 * n
    src = torch.randint(0, n, (e,), device=dev, generator=g)
    dst = torch.randint(0, n, (e,), device=dev, generator=g)
    tc = DenseClosure(src, dst, n, device=dev)
    cntb = torch.zeros(1, dtype=torch.int64, device=dev)
    for v in (0, 1, 2, 3):
        dt = timed(lambda: _ext.ops().tc_step(tc.A, tc.T, tc.T2, cntb, v), 3)
        out[f"closure_step_v{v}"] = {"n": n, "ms": dt * 1e3, "TOPs_int8": 2.0 * tc.npad ** 3 / dt / 1e12}
    # ALS half-sweep
    m, nn, k = (int(x) for x in a.als.split(","))
    als = ALS(ALSConfig(m=m, n=nn, k=k, seed=1), device=dev)
    dt = timed(als.step, 3)
    out["als_sweep"] = {"m": m, "n": nn, "k": k, "ms": dt * 1e3,
                        "GEMM_TFLOPs": 2 * 2.0 * m * nn * k / dt / 1e12, "rmse": als.rmse()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
