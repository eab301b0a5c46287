"""Candidate-pruned K2 diagnostics: per filtered iteration, the distribution of the
128-centre chunks each tile streams (nch = ceil(#{c: nd[a][c] <= R} / 128), R = 2 max ua
over the tile, ua = sqrt(|x - c_a|^2 + tol)), recomputed in torch from the kernel's inputs
(sorted rows, tile table, neighbour lists) just before the K2 launch."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from dalgo.data.synthetic import blobs          # noqa: E402
from dalgo.models.kmeans import KMeans, KMeansConfig   # noqa: E402
from dalgo.ops import kmeans as K               # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=20_000_000)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--no-candidates", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda")
X = blobs(a.rows, 128, a.k, device=dev, dtype=torch.bfloat16, seed=7)
km = KMeans(KMeansConfig(k=a.k, n_iterations=a.iters, seed=42, candidates=not a.no_candidates),
            X, 0, a.rows)
orig = K.assign_rows
stats = []


def lower_bound_quality(X_, cen, idx, post):
    """l written by K2 over the active rows vs the exact second-best distance."""
    n_act = int(post["m_dev"].item())
    r = idx[:n_act].long()
    k = cen.k
    ratios = []
    for s0 in range(0, n_act, 1 << 18):
        rr = r[s0:s0 + (1 << 18)]
        D = torch.cdist(X_[rr, :128].float(), cen.Cq[:k, :128].float())
        two = torch.topk(D, 2, dim=1, largest=False).values
        ratios.append(post["ul"][rr, 1] / two[:, 1].clamp_min(1e-6))
    q = torch.cat(ratios)
    return dict(l_over_second_best_mean=float(q.mean()), l_lt_90pct=float((q < 0.9).float().mean()))


def probe(X_, cen, idx, m, assign, *args, post=None, cand=None, **kw):
    if post is not None and cand is None:
        out = orig(X_, cen, idx, m, assign, *args, post=post, cand=cand, **kw)
        stats.append(dict(active=int(post["m_dev"].item()), **lower_bound_quality(X_, cen, idx, post)))
        return out
    if cand is not None:
        torch.cuda.synchronize()
        n_act = int(post["m_dev"].item())
        T = int(cand.n_tiles.item())
        kpad = cand.kpad
        cs = cand.cstart
        pos = torch.arange(n_act, device=dev)
        c = torch.searchsorted(cs, pos, right=True) - 1
        tiles_per = (cs[1:] - cs[:-1] + K.CAND_TILE - 1) // K.CAND_TILE
        toff = torch.cumsum(tiles_per, 0) - tiles_per
        tid = toff[c] + (pos - cs[c]) // K.CAND_TILE
        r = cand.rows[:n_act].long()
        tol = float(post["tol"].item())
        u = torch.empty(n_act, device=dev)
        for s0 in range(0, n_act, 1 << 22):
            rr = r[s0:s0 + (1 << 22)]
            cc = c[s0:s0 + (1 << 22)]
            xd = X_[rr, :128].float() - cen.Cq[cc, :128].float()
            u[s0:s0 + (1 << 22)] = (xd.pow(2).sum(1) + tol).sqrt()
        umax = torch.zeros(T, device=dev).scatter_reduce(0, tid, u, "amax", include_self=True)
        R = 2 * umax
        tcl = cand.tiles.view(-1, 4)[:T, 0].long()
        nd = cand.nd.view(-1, kpad)[tcl]
        nc = torch.searchsorted(nd, R[:, None], right=True)[:, 0]
        nsub = (nc + 127) // 128
        qs = torch.quantile(nsub.float(), torch.tensor([0.1, 0.5, 0.9, 0.99], device=dev))
        stats.append(dict(active=n_act, tiles=T, chunks=int(nsub.sum()),
                          fraction_of_dense=float(nsub.sum()) / (T * kpad / 128),
                          fraction_of_full_pass=float(nsub.sum()) * K.CAND_TILE * 128
                          / (X_.shape[0] * kpad),
                          nchunks_p10_50_90_99=[float(v) for v in qs],
                          R_median=float(R.median()), u_median=float(u.median()),
                          tile_fill=n_act / (T * K.CAND_TILE)))
    out = orig(X_, cen, idx, m, assign, *args, post=post, cand=cand, **kw)
    if cand is not None:
        stats[-1].update(lower_bound_quality(X_, cen, idx, post))
    return out


K.assign_rows = probe
for it in range(a.iters):
    km.step()
print(json.dumps(stats, indent=1))
