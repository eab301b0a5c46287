"""K1 launch-shape probe at a per-rank share: time lr_grad (atomic epilogue, fused update
tail on one rank) for several workgroup targets / fine-claim thresholds with HIP events."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from dalgo.ops import lr as L                    # noqa: E402
from dalgo.ops import random as R                # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_250_000)
ap.add_argument("--dim", type=int, default=1024)
ap.add_argument("--iters", type=int, default=300)
ap.add_argument("--tbs", default="192,256,320,384,512")
ap.add_argument("--fgs", default="0,8")
ap.add_argument("--reps", type=int, default=1)
a = ap.parse_args()
dev = torch.device("cuda")
X = torch.empty((a.rows, a.dim), dtype=torch.bfloat16, device=dev)
R.philox_fill_(X, D=a.dim, seed=1, stream=3, dist=R.NORMAL, a=0.0, b=1.0)
y = (torch.rand(a.rows, device=dev) > 0.5).float()
W = torch.zeros((1, a.dim + 1), device=dev)
seg = torch.tensor([0, a.rows], dtype=torch.int64, device=dev)
G = torch.zeros_like(W)
C = torch.zeros(1, device=dev)
cnt = torch.zeros(1, dtype=torch.float64, device=dev)
res = {}
for rep in range(a.reps):
  for tb in [int(v) for v in a.tbs.split(",")]:
    for fg in [int(v) for v in a.fgs.split(",")]:
        def run(t):
            L.lr_grad(X, y, W, seg, D=a.dim, seed=7, step=t, frac=0.1, G=G, C=C,
                      target_blocks=tb, fine_groups=fg, g_is_zero=True,
                      tail=dict(mode=0, reg=0, eta=0.01, lam=0.0, reg_alpha=0.0, count_acc=cnt, xg=None))
        for t in range(20):
            run(t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(a.iters):
            run(100 + t)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(f"tb{tb}_fg{fg}", []).append(round(e0.elapsed_time(e1) / a.iters * 1000, 2))
print(json.dumps(res))
