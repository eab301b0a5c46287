"""K8 fused update / synchronisation rules (csrc/kernels/sync_update.hip).

Modes mirror the reference's driver-side NumPy updates (see the kernel header
for file:line citations). All rules act in place on f32 model tensors shaped
``[rows, ld]``; the first ``n`` columns are updated.
"""
from __future__ import annotations

import torch

from dalgo.ops import _ext

SSGD, GD_SUM, LOCAL_MEAN, LOCAL_ELASTIC, AVERAGE, BMUF, ELASTIC_CENTER = range(7)
REG = {"none": 0, "l2": 1, "l1": 2, "elastic_net": 3}


def _reg_grad(w, reg: int, a: float):
    if reg == 1:
        return w
    if reg == 2:
        return torch.sign(w)
    if reg == 3:
        return a * torch.sign(w) + (1 - a) * w
    return torch.zeros_like(w)


def sync_update(W: torch.Tensor, mode: int, *, n: int | None = None, G=None, C=None, center=None,
                S=None, Dl=None, count_acc=None, reg: str | int = "none", eta: float = 0.0, lam: float = 0.0,
                alpha: float = 0.0, reg_alpha: float = 0.0, mu: float = 0.0, zeta: float = 0.0,
                beta: float = 0.0, inv_p: float = 1.0, zero_grad: bool = False) -> torch.Tensor:
    """One K8 launch. ``zero_grad``: the gradient-consuming modes (SSGD, GD, local
    mean/elastic) leave G and C zeroed, ready for the next atomic-epilogue K1."""
    W2 = W if W.dim() == 2 else W.view(1, -1)
    n = W2.shape[1] if n is None else int(n)
    reg_i = REG[reg] if isinstance(reg, str) else int(reg)
    if W2.is_cuda:
        Gv = None if G is None else (G if G.dim() == 2 else G.view(1, -1))
        _ext.ops().sync_update(W2, Gv, None if C is None else C.reshape(-1),
                               None if center is None else center.reshape(-1),
                               None if S is None else S.reshape(-1),
                               None if Dl is None else Dl.reshape(-1), count_acc, n, int(mode), reg_i,
                               float(eta), float(lam), float(alpha), float(reg_alpha), float(mu),
                               float(zeta), float(beta), float(inv_p), bool(zero_grad))
        return W
    # ---- CPU reference (same math, W's dtype)
    if count_acc is not None:
        count_acc += float(C.reshape(-1).double().sum())
    w = W2[:, :n]
    if mode == SSGD:
        c = C.reshape(-1, 1).to(w.dtype)
        g = torch.where(c > 0, G.view(W2.shape[0], -1)[:, :n] / c.clamp_min(1e-30),
                        torch.zeros_like(w))
        w -= eta * (g + lam * _reg_grad(w, reg_i, reg_alpha))
    elif mode == GD_SUM:
        w -= eta * G.view(W2.shape[0], -1)[:, :n]
    elif mode == LOCAL_MEAN:
        c = C.reshape(-1, 1).to(w.dtype)
        g = torch.where(c > 0, G.view(W2.shape[0], -1)[:, :n] / c.clamp_min(1e-30),
                        torch.zeros_like(w))
        w -= eta * g
    elif mode == LOCAL_ELASTIC:
        c = C.reshape(-1, 1).to(w.dtype)
        g = torch.where(c > 0, G.view(W2.shape[0], -1)[:, :n] / c.clamp_min(1e-30),
                        torch.zeros_like(w))
        w.copy_(w - eta * g - alpha * (w - center.reshape(1, -1)[:, :n]))
    elif mode == AVERAGE:
        w.copy_(S.reshape(1, -1)[:, :n] * inv_p)
    elif mode == BMUF:
        wavg = S.reshape(1, -1)[:, :n] * inv_p
        d = Dl.reshape(1, -1)[:, :n]
        d.copy_(mu * d + zeta * (wavg - w))
        w += d
    elif mode == ELASTIC_CENTER:
        w.copy_((1 - beta) * w + beta * (S.reshape(1, -1)[:, :n] * inv_p))
    else:
        raise ValueError(f"unknown update mode {mode}")
    if zero_grad and G is not None and mode in (SSGD, GD_SUM, LOCAL_MEAN, LOCAL_ELASTIC):
        G.zero_()
        if C is not None:
            C.zero_()
    return W


def rows_sum(W: torch.Tensor, out: torch.Tensor, n: int | None = None) -> torch.Tensor:
    """out[:n] = sum over rows of W[:, :n] (fixed order)."""
    n = W.shape[1] if n is None else int(n)
    if W.is_cuda:
        _ext.ops().rows_sum(W, n, out)
        return out
    out.view(-1)[:n] = W[:, :n].sum(dim=0)
    return out


def rows_broadcast(W: torch.Tensor, src: torch.Tensor, n: int | None = None) -> torch.Tensor:
    """W[r, :n] = src[:n] for every row r (reset local models to the global one)."""
    n = W.shape[1] if n is None else int(n)
    if W.is_cuda:
        _ext.ops().rows_broadcast(W, n, src.reshape(-1))
        return W
    W[:, :n] = src.reshape(1, -1)[:, :n]
    return W
