"""Per-iteration phase split of the k-means job (BASELINE config #4 shape): the same data
and model as dalgo.apps.jobs.kmeans_job, with a PhaseTimer (HIP events around centres /
filter / assign / accumulate / update) on a second run after a discarded first one.

usage: python bench/probes/km_phase_split.py [--noise 4] [--rows N] [--dense auto]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--dense", default="auto")
    a = ap.parse_args()
    from dalgo.apps.jobs import reserve_pool
    from dalgo.data.synthetic import blobs
    from dalgo.models.kmeans import KMeans, KMeansConfig
    from dalgo.utils.obs import PhaseTimer
    dev = torch.device("cuda")
    reserve_pool(dev, 48.0)
    X = blobs(a.rows, 128, 1024, row_range=(0, a.rows), device=dev, dtype=torch.bfloat16, seed=7,
              noise=a.noise)
    for rep in range(2):
        km = KMeans(KMeansConfig(k=1024, n_iterations=a.iters, seed=1, dense=a.dense), X, 0, a.rows)
        km.timer = PhaseTimer(dev)
        its = []
        for _ in range(a.iters):
            km.step()
            its.append(km.timer.take())
        torch.cuda.synchronize()
        if rep:
            out = []
            for recs in its:
                ph = {}
                for name, s, e in recs:
                    ph[name] = round(ph.get(name, 0.0) + s.elapsed_time(e), 3)
                out.append(ph)
            print(json.dumps({"noise": a.noise, "dense": a.dense, "phases_ms": out,
                              "active": km.active_history, "moved": km.changed_history,
                              "dense_rows": km.dense_history}), flush=True)
        del km


if __name__ == "__main__":
    main()
