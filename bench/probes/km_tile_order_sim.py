"""CPU estimate of the candidate K2's chunk count per tile when a cluster's active rows are
ordered by their distance to the cluster centre (so a tile's R = 2 max u covers similar
rows) instead of by row id (a tile's R then approaches the cluster's largest distance).

Runs exact Lloyd iterations on a 1M-row sample of the benchmark's blob data, takes the
Hamerly-active rows of each iteration, and for a job of --scale_rows rows (100M: ~256x
more rows per cluster than the sample) models a tile of 256 rows as a quantile range of
its cluster's distance distribution:
  row order:    every tile's max distance ~ the cluster's (1 - 1/256) quantile
  sorted order: tile i of T has max distance = the (i + 1) / T quantile
Chunks per tile = 1 + #{chunk j >= 1 of the cluster's neighbour list whose first centre
distance is <= 2 max}. Prints the mean chunks per tile (of 8) for both orders.
"""
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dalgo.data.synthetic import blobs               # noqa: E402
from dalgo.models.kmeans import sample_rows          # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000)
ap.add_argument("--scale_rows", type=int, default=100_000_000)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
torch.set_num_threads(8)
X = blobs(a.rows, 128, a.k, dtype=torch.float32, seed=7)
x2 = (X * X).sum(1)
C = X[torch.from_numpy(sample_rows(a.rows, a.k, 42))].clone()
CH = 128


def top2(C):
    best = torch.empty(a.rows)
    sec = torch.empty(a.rows)
    arg = torch.empty(a.rows, dtype=torch.long)
    c2 = (C * C).sum(1)
    for s in range(0, a.rows, 1 << 17):
        e = min(a.rows, s + (1 << 17))
        dd = (x2[s:e, None] - 2 * X[s:e] @ C.T + c2[None]).clamp_min(0).sqrt()
        v, i = torch.topk(dd, 2, dim=1, largest=False)
        best[s:e], sec[s:e], arg[s:e] = v[:, 0], v[:, 1], i[:, 0]
    return best, sec, arg


d1, d2, arg = top2(C)
u, lo, asg = d1.clone(), d1.clone(), arg.clone()
mult = a.scale_rows / a.rows
out = {}
for it in range(2, a.iters + 1):
    S = torch.zeros_like(C).index_add_(0, arg, X)
    cnt = torch.bincount(arg, minlength=a.k).float()
    Cn = C.clone()
    Cn[cnt > 0] = S[cnt > 0] / cnt[cnt > 0, None]
    delta = (Cn - C).norm(dim=1)
    cc = torch.cdist(Cn, Cn)
    cc.fill_diagonal_(float("inf"))
    s_half = 0.5 * cc.min(dim=1).values
    cc.fill_diagonal_(0.0)
    nd = torch.sort(cc, dim=1).values
    thr = nd[:, CH::CH]                                  # first distance of chunks 1..7
    ub = u + delta[asg]
    act = ~(ub < torch.maximum(s_half[asg], lo - float(delta.max())))
    # distance of each active row to its (previous) cluster's new centre
    da = (X - Cn[asg]).norm(dim=1)
    tot = {"row_order": 0.0, "sorted": 0.0}
    tiles = 0.0
    for c in range(a.k):
        m = act & (asg == c)
        n_c = int(m.sum()) * mult
        if n_c < 1:
            continue
        T = max(1, int(np.ceil(n_c / 256)))
        q = torch.sort(da[m]).values.numpy()
        qq = lambda f: q[min(len(q) - 1, int(np.floor(f * len(q))))]
        th = thr[c].numpy()
        r_row = 2 * qq(1 - 1 / 256) if T > 1 else 2 * q[-1]
        tot["row_order"] += T * (1 + int((th <= r_row).sum()))
        for i in range(T):
            tot["sorted"] += 1 + int((th <= 2 * qq(min(1.0, (i + 1) / T) - 1e-9)).sum())
        tiles += T
    res = {"active": float(act.float().mean()),
           "chunks_per_tile_row_order": tot["row_order"] / tiles,
           "chunks_per_tile_sorted": tot["sorted"] / tiles}
    out[f"iteration_{it}"] = res
    print(it, json.dumps(res), flush=True)
    d1, d2, arg = top2(Cn)
    u = torch.where(act, d1, ub)
    lo = torch.where(act, d2, lo - float(delta.max()))
    asg = torch.where(act, arg, asg)
    C = Cn
print(json.dumps(out))
