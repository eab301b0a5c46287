#!/usr/bin/env python3
"""Eager launches vs hipGraph replay of whole LR-family training steps (1 GPU).

A step is K1 + K8 (SSGD / GD), K1 + 2 x K8 + row sum (EASGD) or a 5-local-step
MA / BMUF round (rows broadcast, 5 x (K1 + K8), row sum, K8): small problems are
launch bound, which the captured step (ParallelSGD.graph, DALGO_GRAPH=1) removes.
Prints one JSON line per (algo, problem): us/step eager and replayed.

Run: python bench/graph_replay.py [--steps 300]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalgo.data.datasets import synthetic_logistic  # noqa: E402
from dalgo.models.localsgd import ParallelSGD, SGDConfig  # noqa: E402
from dalgo.parallel import runtime  # noqa: E402
from dalgo.parallel.sharding import make_layout  # noqa: E402


def time_steps(m: ParallelSGD, steps: int) -> float:
    m.fit(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.fit(steps)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rt = runtime.init(device="cuda")
    problems = [("breast-cancer-shape 398x30 f32, 4 workers", 398, 30, torch.float32, 4),
                ("100k x 256 bf16, 4 workers", 100_000, 256, torch.bfloat16, 4),
                ("1.25M x 1024 bf16, 1 worker", 1_250_000, 1024, torch.bfloat16, 1)]
    lines = []
    for name, n, d, dt, P in problems:
        data = synthetic_logistic(n, d, device=rt.device, dtype=dt)
        lay = make_layout(n, P, 1, 0, spark_compatible=False)
        for algo in ("ssgd", "gd", "ma", "bmuf", "easgd"):
            if P == 1 and algo != "ssgd":
                continue
            res = {}
            for graph in (False, True):
                cfg = SGDConfig(algo=algo, n_workers=P, eval_every=0, n_iterations=a.steps,
                                eta=0.1 if algo != "gd" else 1e-4)
                m = ParallelSGD(cfg, data, lay, rt)
                m.graph = graph
                res["graph" if graph else "eager"] = time_steps(m, a.steps)
            line = dict(problem=name, algo=algo, eager_us_per_step=round(res["eager"], 2),
                        graph_us_per_step=round(res["graph"], 2),
                        speedup=round(res["eager"] / res["graph"], 3))
            print(json.dumps(line), flush=True)
            lines.append(line)
    if a.out:
        with open(a.out, "w") as f:
            for line in lines:
                f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
