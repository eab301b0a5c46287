"""CPU simulation of exact Lloyd k-means on the bench's blob data (smaller n), measuring how
much distance work each exact filter leaves per iteration (design probe for the drift-aware
candidate K2; not part of the library). Prints per iteration: Hamerly-active rows, and the
centre candidates per active row under the Exponion ball (|c - c_a| < 2 u_new), the drift
bound (l - delta_c < u_new) and both, plus the tile-granularity union (256 rows of one
cluster)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dalgo.data.synthetic import blobs  # noqa: E402
from dalgo.models.kmeans import sample_rows  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
noise = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
k, d = 1024, 128
torch.set_num_threads(8)
X = blobs(n, d, k, seed=7, noise=noise).float()
ids = sample_rows(n, k, 1)
C = X[torch.from_numpy(ids)].clone()
xx = (X * X).sum(1)


def dists(C):
    out = torch.empty(n, k)
    cc = (C * C).sum(1)
    for s in range(0, n, 1 << 17):
        e = min(n, s + (1 << 17))
        out[s:e] = (xx[s:e, None] - 2 * X[s:e] @ C.T + cc[None]).clamp_min(0).sqrt()
    return out


def update(C, a):
    S = torch.zeros(k, d).index_add_(0, a, X)
    cnt = torch.bincount(a, minlength=k).float()
    return torch.where(cnt[:, None] > 0, S / cnt.clamp_min(1)[:, None], C)


D = dists(C)
top = D.topk(2, dim=1, largest=False)
a = top.indices[:, 0]
u, l = top.values[:, 0], top.values[:, 1]
for it in range(2, 7):
    Cn = update(C, a)
    delta = (Cn - C).norm(dim=1)
    maxd = float(delta.max())
    cc = torch.cdist(Cn, Cn)
    cc.fill_diagonal_(float("inf"))
    s = 0.5 * cc.min(1).values
    act = (u + delta[a]) >= torch.maximum(s[a], l - maxd)
    Dn = dists(Cn)
    un = Dn.gather(1, a[:, None])[:, 0]
    act2 = act & (un >= torch.maximum(s[a], l - maxd))
    ia = torch.nonzero(act).flatten()
    ca = a[ia]
    # per active row: candidates c != a
    ball = cc[ca] < 2 * un[ia, None]                        # [m, k]
    drift = (l[ia, None] - delta[None, :]) < un[ia, None]
    drift[torch.arange(ia.numel()), ca] = False
    both = ball & drift
    # tiles of 256 rows of one cluster (rows sorted by cluster)
    order = torch.argsort(ca, stable=True)
    cs = ca[order]
    tiles_u, tiles_b = [], []
    pos = 0
    bounds = torch.nonzero(torch.diff(cs, prepend=torch.tensor([-1]))).flatten().tolist() + [cs.numel()]
    for i in range(len(bounds) - 1):
        for t0 in range(bounds[i], bounds[i + 1], 256):
            t1 = min(bounds[i + 1], t0 + 256)
            rows = order[t0:t1]
            tiles_u.append(int(both[rows].any(0).sum()))
            tiles_b.append(int(ball[rows].any(0).sum()))
    tiles_u = np.array(tiles_u)
    tiles_b = np.array(tiles_b)
    chunks = np.ceil((tiles_u + 1) / 128)                   # + own centre
    chunks_b = np.ceil((tiles_b + 1) / 128)
    newtop = Dn.topk(2, dim=1, largest=False)
    a_new = newtop.indices[:, 0]
    moved = int((a_new != a).sum())
    print(f"it {it}: active {act.float().mean():.3f} (exact-u {act2.float().mean():.3f}) moved {moved / n:.4f} "
          f"maxd {maxd:.1f} | cand/row: ball {ball.sum(1).float().mean():.1f} drift {drift.sum(1).float().mean():.1f} "
          f"both {both.sum(1).float().mean():.1f} | tile union both {tiles_u.mean():.1f} -> chunk work "
          f"{(chunks * 128).mean() / k:.3f} of dense; ball-only chunk work {(chunks_b * 128).mean() / k:.3f}",
          flush=True)
    C, a = Cn, a_new
    u, l = newtop.values[:, 0], newtop.values[:, 1]
