"""Datasets: the reference's breast-cancer split and sharded synthetic generators.

* :func:`breast_cancer` — ``load_breast_cancer`` + ``train_test_split(test_size=0.3,
  random_state=0, shuffle=True)`` exactly as optimization/ssgd.py:71-76 (398 train /
  171 test, 30 unnormalised features). The reference appends a ones column and
  the label (ssgd.py:83-84); here the bias is handled inside the kernels
  (``has_bias``) and labels are a separate f32 vector.
* :func:`synthetic_logistic` — rows [lo, hi) of a global N x D logistic-model
  dataset generated ON DEVICE by the Philox fill kernel: X ~ U[-1, 1), planted
  w* ~ N(0, 1) * scale / sqrt(D/3), y ~ Bernoulli(sigmoid(x.w* + b*)). Every value is
  keyed by its global index, so any sharding reproduces the same global data.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from dalgo.ops import random as drandom
from dalgo.ops.lr import padded_cols
from dalgo.utils import philox


@dataclass
class LRData:
    X_train: torch.Tensor   # [n_local, D] (row stride padded to 16 B)
    y_train: torch.Tensor   # [n_local] f32
    X_test: torch.Tensor
    y_test: torch.Tensor
    D: int
    n_train_global: int
    row_offset: int = 0     # global index of local train row 0


def _padded(n, D, dtype, device):
    ld = padded_cols(D, dtype)
    return torch.zeros((n, ld), dtype=dtype, device=device)[:, :D]


def breast_cancer(device="cpu", dtype=torch.float32, row_range: tuple[int, int] | None = None,
                  test_size: float = 0.3, random_state: int = 0) -> LRData:
    from sklearn.datasets import load_breast_cancer
    from sklearn.model_selection import train_test_split
    X, y = load_breast_cancer(return_X_y=True)
    X_train, X_test, y_train, y_test = train_test_split(
        X, y, test_size=test_size, random_state=random_state, shuffle=True)
    n = X_train.shape[0]
    lo, hi = row_range if row_range is not None else (0, n)
    D = X.shape[1]
    Xtr = _padded(hi - lo, D, dtype, device)
    Xtr.copy_(torch.from_numpy(X_train[lo:hi]).to(dtype))
    Xte = _padded(X_test.shape[0], D, dtype, device)
    Xte.copy_(torch.from_numpy(X_test).to(dtype))
    return LRData(Xtr, torch.from_numpy(y_train[lo:hi]).float().to(device), Xte,
                  torch.from_numpy(y_test).float().to(device), D, n, lo)


def planted_model(D: int, seed: int, scale: float = 3.0) -> np.ndarray:
    """w* (D+1 entries, last = bias) of the synthetic logistic model."""
    u = philox.uniform01(seed, 0x5EED, np.arange(2 * (D + 1)))
    u1 = np.maximum(u[0::2], 1e-7)
    g = np.sqrt(-2.0 * np.log(u1)) * np.cos(2 * np.pi * u[1::2])
    w = g * (scale / np.sqrt(D / 3.0))
    w[-1] = 0.1 * g[-1]
    return w.astype(np.float32)


def synthetic_logistic(n_rows: int, D: int, *, row_range: tuple[int, int] | None = None,
                       n_test: int = 0, device="cpu", dtype=torch.bfloat16, seed: int = 1234,
                       chunk_rows: int = 1 << 20) -> LRData:
    lo, hi = row_range if row_range is not None else (0, n_rows)
    w_star = torch.from_numpy(planted_model(D, seed)).to(device)

    def make(n, off, stream_x, stream_y):
        X = _padded(n, D, dtype, device)
        y = torch.empty(n, dtype=torch.float32, device=device)
        from dalgo.parallel import runtime
        for s in range(0, n, chunk_rows):
            runtime.heartbeat()   # long generation is progress (stall watchdog)
            e = min(n, s + chunk_rows)
            base = X.as_strided((e - s, X.stride(0)), (X.stride(0), 1), X.storage_offset() + s * X.stride(0))
            drandom.philox_fill_(base, D=D, row_offset=off + s, seed=seed, stream=stream_x,
                                 dist=drandom.UNIFORM, a=-1.0, b=1.0)
            z = X[s:e].float() @ w_star[:D] + w_star[D]
            u = torch.empty(e - s, dtype=torch.float32, device=device)
            drandom.philox_fill_(u.view(-1, 1), D=1, row_offset=off + s, seed=seed,
                                 stream=stream_y, dist=drandom.UNIFORM, a=0.0, b=1.0)
            y[s:e] = (u < torch.sigmoid(z)).float()
        return X, y

    Xtr, ytr = make(hi - lo, lo, 1, 2)
    if n_test > 0:
        Xte, yte = make(n_test, 0, 3, 4)
    else:
        Xte, yte = Xtr[:0], ytr[:0]
    return LRData(Xtr, ytr, Xte, yte, D, n_rows, lo)
