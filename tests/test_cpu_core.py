"""CPU unit tests: Philox mirror, sharding, update rules, data pipeline."""
import numpy as np
import pytest
import torch

from dalgo.ops import update as U
from dalgo.parallel.sharding import even_slices, make_layout, spark_slices
from dalgo.utils import philox


def test_philox_known_answer():
    # Random123 known-answer vector for Philox4x32-10, counter=0, key=0
    r = philox.philox4x32_10(np.uint32([0]), np.uint32([0]), np.uint32([0]), np.uint32([0]), 0, 0)
    assert [int(x[0]) for x in r] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_philox_uniform_and_bernoulli_rate():
    idx = np.arange(200_000)
    u = philox.uniform01(3, 9, idx)
    assert 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
    m = philox.bernoulli_mask(42, 5, idx, 0.1)
    assert abs(m.mean() - 0.1) < 0.005
    # index-keyed: any sub-range reproduces the same draws
    assert np.array_equal(philox.draw_u32(1, 2, idx[1000:2000]), philox.draw_u32(1, 2, idx)[1000:2000])


def test_spark_slices_breast_cancer():
    # sc.parallelize(398 rows, 4) -> 99/99/99/101
    s = spark_slices(398, 4)
    assert [b - a for a, b in s] == [99, 99, 99, 101]
    assert s[0][0] == 0 and s[-1][1] == 398
    assert [b - a for a, b in even_slices(10, 3)] == [3, 3, 4]


def test_layout_ranks_partition_workers():
    lay0 = make_layout(398, 4, 2, 0)
    lay1 = make_layout(398, 4, 2, 1)
    assert (lay0.row_lo, lay0.row_hi, lay1.row_lo, lay1.row_hi) == (0, 198, 198, 398)
    assert lay1.local_segments() == [0, 99, 200]
    with pytest.raises(ValueError):
        make_layout(398, 3, 2, 0)


def test_update_rules_match_reference_formulas():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(1, 31, generator=g, dtype=torch.float64)
    G = torch.randn(1, 31, generator=g, dtype=torch.float64)
    C = torch.tensor([7.0], dtype=torch.float64)
    # SSGD with l2 (ssgd.py:105)
    w1 = w.clone()
    U.sync_update(w1, U.SSGD, G=G, C=C, reg="l2", eta=0.1, lam=0.5)
    assert torch.allclose(w1, w - 0.1 * (G / 7 + 0.5 * w))
    # BMUF (bmuf.py:111-114)
    S = torch.randn(31, generator=g, dtype=torch.float64)
    D = torch.randn(31, generator=g, dtype=torch.float64)
    w2, D2 = w.clone(), D.clone()
    U.sync_update(w2, U.BMUF, S=S, Dl=D2, mu=0.9, zeta=0.1, inv_p=0.25)
    dref = 0.9 * D + 0.1 * (S / 4 - w[0])
    assert torch.allclose(D2, dref) and torch.allclose(w2[0], w[0] + dref)
    # EASGD centre (easgd.py:106)
    w3 = w.clone()
    U.sync_update(w3, U.ELASTIC_CENTER, S=S, beta=0.04, inv_p=0.25)
    assert torch.allclose(w3[0], 0.96 * w[0] + 0.04 * S / 4)


def test_breast_cancer_split():
    from dalgo.data.datasets import breast_cancer
    d = breast_cancer()
    assert d.X_train.shape == (398, 30) and d.X_test.shape == (171, 30)
    assert d.X_train.stride(0) % 2 == 0   # 16-B padded rows


def test_lr_grad_device_step_counter_cpu():
    """K1's graph-replay stream (step + step_mul * step_dev) selects the same rows as
    the plain step argument (CPU reference path)."""
    from dalgo.ops import lr as L
    g = torch.Generator().manual_seed(3)
    X = torch.rand((3000, 17), generator=g, dtype=torch.float64)
    y = (torch.rand(3000, generator=g) < 0.5).double()
    W = torch.randn(1, 18, generator=g, dtype=torch.float64)
    seg = torch.tensor([0, 3000])
    kw = dict(D=17, seed=42, frac=0.1)
    G1, C1 = L.lr_grad(X, y, W, seg, step=2 + 5 * 7, **kw)
    G2, C2 = L.lr_grad(X, y, W, seg, step=2, step_dev=torch.tensor([7]), step_mul=5, **kw)
    assert torch.equal(C1, C2) and torch.equal(G1, G2)
