#!/usr/bin/env python3
"""A/B of the k-means assign kernel variants (interleaved rounds, one process)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalgo.data.synthetic import blobs  # noqa: E402
from dalgo.ops import kmeans as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X = K.prepare_points(blobs(a.rows, a.dim, a.k, device=dev, dtype=torch.bfloat16, seed=3))
    C0 = X[torch.randperm(a.rows, device=dev)[: a.k]].float()
    cen = K.make_centers(C0, torch.bfloat16, dev)
    vs = [int(v) for v in a.variants.split(",")]
    ref = K.assign(X, cen, variant=0).clone()
    for v in vs:
        out = K.assign(X, cen, variant=v)
        torch.cuda.synchronize()
        print(json.dumps({"variant": v, "mismatch": int((out != ref).sum().item())}))
    res = {v: [] for v in vs}
    for _ in range(a.rounds):
        for v in vs:
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                K.assign(X, cen, out=ref, variant=v)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t) / 3)
    fl = 2.0 * a.rows * a.k * a.dim
    for v, ts in sorted(res.items(), key=lambda kv: min(kv[1])):
        print(json.dumps({"variant": v, "ms": min(ts) * 1e3, "TFLOPs": fl / min(ts) / 1e12}))


if __name__ == "__main__":
    main()
