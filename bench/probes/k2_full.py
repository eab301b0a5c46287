"""K2 full pass alone (bf16 100M x 128, k = 1024, the k-means job's data): device time per
pass (HIP events, best of --reps) and PF/s; for PMC runs under rocprofv3."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.data.synthetic import blobs          # noqa: E402
from dalgo.ops import kmeans as K               # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--noise", type=float, default=1.0)
a = ap.parse_args()
dev = torch.device("cuda")
X = K.prepare_points(blobs(a.rows, 128, a.k, device=dev, dtype=torch.bfloat16, seed=7, noise=a.noise))
g = torch.Generator(device="cpu").manual_seed(1)
C0 = X[torch.randperm(a.rows, generator=g)[: a.k].to(dev), :128].float()
cen = K.make_centers(C0, torch.bfloat16, dev)
out = torch.empty(a.rows, dtype=torch.int32, device=dev)
ts = []
for _ in range(a.reps + 1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    K.assign(X, cen, out=out)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
best = min(ts[1:])
print(json.dumps({"rows": a.rows, "k": a.k, "ms": best, "all_ms": ts,
                  "pflops": 2.0 * a.rows * a.k * 128 / (best / 1e3) / 1e15,
                  "lib": os.environ.get("DALGO_EXT_LIB", "in-tree")}), flush=True)
