"""CPU simulation of the bound-filtered Lloyd iterations with the bounds carried as the
kernels carry them (u, l per row; skipped rows: u += delta_a, l -= maxd; re-assigned rows:
u exact, l = min(second best among the streamed centres, ball bound nd_first - u,
drift bound l_old - max delta of the drift-pruned centres)) at 256-row tile granularity
(rows sorted by cluster), 128-centre chunks. Design probe for the drift-aware candidate
K2 (not part of the library). usage: n noise top2_first(0/1) drift(0/1)"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dalgo.data.synthetic import blobs  # noqa: E402
from dalgo.models.kmeans import sample_rows  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
noise = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top2_first = int(sys.argv[3]) if len(sys.argv) > 3 else 1
use_drift = int(sys.argv[4]) if len(sys.argv) > 4 else 1
TILE = int(sys.argv[5]) if len(sys.argv) > 5 else 256
FRAC = float(sys.argv[6]) if len(sys.argv) > 6 else 1.0      # drift threshold = FRAC * tau_T
DENSE2 = int(sys.argv[7]) if len(sys.argv) > 7 else 1        # iteration 2 dense (exact top-2)
CH = 128
k, d = 1024, 128
torch.set_num_threads(8)
X = blobs(n, d, k, seed=7, noise=noise).float()
C = X[torch.from_numpy(sample_rows(n, k, 1))].clone()
xx = (X * X).sum(1)


def dists(C, rows=None):
    Xr = X if rows is None else X[rows]
    xr = xx if rows is None else xx[rows]
    m = Xr.shape[0]
    out = torch.empty(m, k)
    cc = (C * C).sum(1)
    for s in range(0, m, 1 << 17):
        e = min(m, s + (1 << 17))
        out[s:e] = (xr[s:e, None] - 2 * Xr[s:e] @ C.T + cc[None]).clamp_min(0).sqrt()
    return out


def update(C, a):
    S = torch.zeros(k, d).index_add_(0, a, X)
    cnt = torch.bincount(a, minlength=k).float()
    return torch.where(cnt[:, None] > 0, S / cnt.clamp_min(1)[:, None], C)


D = dists(C)
top = D.topk(2, dim=1, largest=False)
a = top.indices[:, 0].clone()
u = top.values[:, 0].clone()
l = (top.values[:, 1] if top2_first else top.values[:, 0]).clone()
del D
tot_work = 1.0
for it in range(2, 6):
    Cn = update(C, a)
    delta = (Cn - C).norm(dim=1)
    maxd = float(delta.max())
    cc = torch.cdist(Cn, Cn)
    cc.fill_diagonal_(float("inf"))
    s = 0.5 * cc.min(1).values
    act = (u + delta[a]) >= torch.maximum(s[a], l - maxd)
    # skipped rows
    sk = ~act
    u[sk] += delta[a[sk]]
    l[sk] -= maxd
    ia = torch.nonzero(act).flatten()
    ca = a[ia]
    order = torch.argsort(ca, stable=True)
    ia, ca = ia[order], ca[order]
    Dn = dists(Cn, ia)                                     # [m, k] exact
    un = Dn.gather(1, ca[:, None])[:, 0]
    ccd = cc.clone()
    ccd.fill_diagonal_(0.0)
    m = ia.numel()
    new_a = ca.clone()
    new_u = un.clone()
    new_l = torch.empty(m)
    work = 0
    bnd = torch.nonzero(torch.diff(ca, prepend=torch.tensor([-1]))).flatten().tolist() + [m]
    for i in range(len(bnd) - 1):
        c0 = int(ca[bnd[i]])
        for t0 in range(bnd[i], bnd[i + 1], TILE):
            t1 = min(bnd[i + 1], t0 + TILE)
            R = 2 * float(un[t0:t1].max())
            inball = ccd[c0] <= R
            if DENSE2 and it == 2:
                inball = torch.ones_like(inball)
            if use_drift and not (DENSE2 and it == 2):
                tau = FRAC * float((l[ia[t0:t1]] - un[t0:t1]).min())
                keep = inball & (delta > tau)
            else:
                keep = inball.clone()
            keep[c0] = True
            nkeep = int(keep.sum())
            work += TILE * (-(-nkeep // CH)) * CH
            Dt = Dn[t0:t1][:, keep]
            ids = torch.nonzero(keep).flatten()
            tt = Dt.topk(min(2, nkeep), dim=1, largest=False)
            new_a[t0:t1] = ids[tt.indices[:, 0]]
            new_u[t0:t1] = tt.values[:, 0]
            sec = tt.values[:, 1] if nkeep > 1 else torch.full((t1 - t0,), float("inf"))
            out_ball = ~inball
            nd_first = float(ccd[c0][out_ball].min()) if out_ball.any() else float("inf")
            lb = torch.minimum(sec, nd_first - un[t0:t1])
            if use_drift and not (DENSE2 and it == 2):
                dp = (~keep) & inball
                dmp = float(delta[dp].max()) if dp.any() else 0.0
                if dp.any():
                    lb = torch.minimum(lb, l[ia[t0:t1]] - dmp)
            new_l[t0:t1] = lb
    # exactness check: the streamed argmin equals the true argmin (ties aside)
    true_a = Dn.argmin(1)
    bad = int(((Dn.gather(1, new_a[:, None])[:, 0] - Dn.gather(1, true_a[:, None])[:, 0]) > 1e-4).sum())
    a[ia] = new_a
    u[ia] = new_u
    l[ia] = new_l
    moved = int((new_a != ca).sum())
    frac_work = work / (n * k)
    tot_work += frac_work
    print(f"it {it}: active {m / n:.3f} moved {moved / n:.4f} maxd {maxd:.1f} streamed work "
          f"{frac_work:.3f} of a full pass (per active row {work / max(m, 1) / k:.3f}); wrong {bad}",
          flush=True)
    C = Cn
print(f"job work (full-pass units, 5 iterations): {tot_work:.3f}")
