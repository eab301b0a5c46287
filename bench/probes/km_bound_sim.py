"""CPU simulation of the bound filter's active fraction per Lloyd iteration (exact f32
distances, no kernels): Hamerly's test (global max centre shift) against the same test
with a per-cluster neighbourhood bound -- for a row of cluster a, the centres closer to
c_a than D moved by at most pmax(a, D) (the largest shift among them), every other
centre is at least D - u from the row, so
    other distances >= max over D of min(l - pmax(a, D), D - u).
D runs over a's sorted centre distances (all of them, or a few list positions).
Bounds are maintained exactly as the filter does (skipped rows drift, active rows get
the exact best / second-best distance).

    python bench/probes/km_bound_sim.py --rows 1000000 --k 1024
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
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--iters", type=int, default=6)
ap.add_argument("--positions", default="all", help="'all' or comma list of list positions")
a = ap.parse_args()
torch.set_num_threads(8)
X = blobs(a.rows, a.d, a.k, dtype=torch.float32, seed=7)
x2 = (X * X).sum(1)
C = X[torch.from_numpy(sample_rows(a.rows, a.k, 42))].clone()


def top2(C):
    best = torch.full((a.rows,), float("inf"))
    sec = torch.full((a.rows,), float("inf"))
    arg = torch.zeros(a.rows, dtype=torch.long)
    c2 = (C * C).sum(1)
    for s in range(0, a.rows, 1 << 17):
        e = min(a.rows, s + (1 << 17))
        dd = (x2[s:e, None] - 2 * X[s:e] @ C.T + c2[None]).clamp_min(0).sqrt()
        v, i = torch.topk(dd, 2, dim=1, largest=False)
        best[s:e], sec[s:e], arg[s:e] = v[:, 0], v[:, 1], i[:, 0]
    return best, sec, arg


def update(arg):
    S = torch.zeros_like(C).index_add_(0, arg, X)
    cnt = torch.bincount(arg, minlength=a.k).float()
    Cn = C.clone()
    nz = cnt > 0
    Cn[nz] = S[nz] / cnt[nz, None]
    return Cn


out = {}
d1, d2, arg = top2(C)
u = {m: d1.clone() for m in ("hamerly", "nbhd")}
lo = {m: d1.clone() for m in ("hamerly", "nbhd")}   # first pass: l = best (as the plain K2)
asg = {m: arg.clone() for m in ("hamerly", "nbhd")}
for it in range(2, a.iters + 1):
    Cn = update(arg)
    delta = (Cn - C).norm(dim=1)
    maxd = float(delta.max())
    cc = torch.cdist(Cn, Cn)
    cc.fill_diagonal_(float("inf"))
    s_half = 0.5 * cc.min(dim=1).values
    cc.fill_diagonal_(0.0)
    nd, nb = torch.sort(cc, dim=1)                       # nd[a, 0] = 0 (a itself)
    pmax = torch.cummax(delta[nb], dim=1).values         # largest shift among positions <= j
    if a.positions == "all":
        pos = torch.arange(1, a.k)
    else:
        pos = torch.tensor([int(p) for p in a.positions.split(",")])
    # near set for D = nd[:, j]: positions < j (shift pmax[:, j - 1]); far: >= D - u
    ndj = nd[:, pos]
    pmj = pmax[:, pos - 1]
    d1, d2, arg = top2(Cn)
    res = {"max_shift": maxd}
    for m in ("hamerly", "nbhd"):
        A = asg[m]
        ub = u[m] + delta[A]
        lb_h = lo[m] - maxd
        bound = torch.maximum(s_half[A], lb_h)
        if m == "nbhd":
            best_lb = torch.full_like(ub, -float("inf"))
            for s in range(0, a.rows, 1 << 16):
                e = min(a.rows, s + (1 << 16))
                Ab = A[s:e]
                cand = torch.minimum(lo[m][s:e, None] - pmj[Ab], ndj[Ab] - ub[s:e, None])
                best_lb[s:e] = cand.max(dim=1).values
            lb = torch.maximum(lb_h, best_lb)
            bound = torch.maximum(bound, lb)
        else:
            lb = lb_h
        act = ~(ub < bound)
        res[m + "_active"] = float(act.float().mean())
        # skipped rows: drifted bounds; active rows: exact
        u[m] = torch.where(act, d1, ub)
        lo[m] = torch.where(act, d2, lb)
        asg[m] = torch.where(act, arg, A)
        assert bool((asg[m] == arg).all()), "bound violated"
    res["moved"] = float((arg != asg["hamerly"]).float().mean())
    out[f"iteration_{it}"] = res
    print(it, json.dumps(res), flush=True)
    C = Cn
print(json.dumps(out))
