"""CPU reference paths of the k-means ops (dalgo/ops/kmeans.py) against explicit numpy
definitions: assign (nearest rounded centre, ties to the lowest id), accumulate (per-cluster
sums / counts), update (empty clusters keep their centre, k-means.py:70-71) and the bound
filter's centre bounds (shift and half the nearest-centre distance).
Reference: machine_learning/k-means.py:20-28 (closestPoint), 55-71 (reduceByKey + update)."""
import numpy as np
import pytest
import torch

from dalgo.ops import kmeans as K


def _data(n, d, k, seed):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g, dtype=torch.float32)
    C = torch.randn(k, d, generator=g, dtype=torch.float32)
    return K.prepare_points(X), C


@pytest.mark.parametrize("d,k", [(5, 3), (16, 7), (100, 33)])
def test_assign_matches_brute_force(d, k):
    X, C = _data(2000, d, k, seed=d + k)
    cen = K.make_centers(C, X.dtype, "cpu")
    mind = torch.empty(X.shape[0], dtype=torch.float32)
    sse = torch.zeros(1, dtype=torch.float64)
    a = K.assign(X, cen, mind=mind, sse=sse).long()
    Xn = X.double().numpy()
    Cn = cen.Cq[:k, :d].double().numpy()
    D = ((Xn[:, None, :] - Cn[None, :, :]) ** 2).sum(-1)
    ref = D.argmin(1)
    # exact f64 scores: any disagreement must be a tie within rounding
    bad = np.nonzero(a.numpy() != ref)[0]
    for i in bad:
        assert abs(D[i, a[i]] - D[i, ref[i]]) <= 1e-9 * max(1.0, D[i, ref[i]])
    assert np.allclose(mind.double().numpy(), D[np.arange(len(ref)), a.numpy()], rtol=1e-5, atol=1e-5)
    assert abs(float(sse) - float(D[np.arange(len(ref)), a.numpy()].sum())) <= 1e-6 * float(sse)


def test_assign_ties_lowest_id():
    X = K.prepare_points(torch.zeros(4, 3))
    C = torch.tensor([[1.0, 0, 0], [0, 1.0, 0], [-1.0, 0, 0]])
    cen = K.make_centers(C, X.dtype, "cpu")
    assert K.assign(X, cen).tolist() == [0, 0, 0, 0]


def test_accumulate_and_update():
    n, d, k = 3000, 10, 6
    X, C = _data(n, d, k, seed=3)
    a = torch.randint(0, k - 1, (n,), generator=torch.Generator().manual_seed(4), dtype=torch.int32)
    DP = K.kmeans_dp(d)
    S = torch.zeros(k * DP, dtype=torch.float64)
    cnt = torch.zeros(k, dtype=torch.int64)
    K.accumulate(X, a, k, DP, S, cnt)
    Xn, an = X.double().numpy(), a.numpy()
    for c in range(k):
        rows = Xn[an == c]
        assert int(cnt[c]) == len(rows)
        assert np.allclose(S.view(k, DP)[c, :d].numpy(), rows.sum(0) if len(rows) else 0.0)
        assert np.all(S.view(k, DP)[c, d:].numpy() == 0)
    # update: cluster k-1 is empty -> keeps its centre; the others become the means
    cen = K.make_centers(C, X.dtype, "cpu")
    old = cen.C.clone()
    shift2 = torch.zeros(1, dtype=torch.float32)
    K.update(cen, S.float(), cnt, shift2)
    for c in range(k):
        want = old[c] if cnt[c] == 0 else S.view(k, DP)[c, :d].float() / float(cnt[c])
        assert torch.allclose(cen.C[c], want, atol=1e-5)
    assert float(shift2) == pytest.approx(float(((cen.C - old) ** 2).sum()), rel=1e-5)
    assert torch.equal(cen.Cq[:k, :d], cen.C.to(cen.Cq.dtype))


def test_centre_bounds_definition():
    k, d = 9, 12
    g = torch.Generator().manual_seed(5)
    now = torch.randn(k, d, generator=g)
    prev = now + 0.1 * torch.randn(k, d, generator=g)
    delta, s = K.centre_bounds(now, prev, k, d)
    a, b = now.double(), prev.double()
    assert bool((delta.double() >= (a - b).norm(dim=1)).all())           # rounded up
    dd = torch.cdist(a, a)
    dd.fill_diagonal_(float("inf"))
    half = 0.5 * dd.min(dim=1).values
    assert bool((s.double() <= half).all())                               # rounded down
    assert torch.allclose(s.double(), half, rtol=1e-5)
    _, s1 = K.centre_bounds(now[:1], prev[:1], 1, d)
    assert float(s1[0]) == float("inf")                                   # no other centre
