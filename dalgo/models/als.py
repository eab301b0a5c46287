"""Distributed ALS matrix decomposition (matrix_computation/matrix_decomposition.py).

Reference (:42-67): R = rand(m,k) rand(n,k)^T, U,V ~ U[0,1); 5 sweeps of
  U_i = (V^T V + lam*n*I)^-1 V^T R_i,:   for every row i   (:52-54, update :24-33)
  V_j = (U^T U + lam*m*I)^-1 U^T R_:,j   for every row j   (:60-62)
then rmse(R, U, V) (:19-21). ("ALS to solve the SVD problem" says the comment at
:50 — it is regularised low-rank factorisation.)

Row-partitioned model parallelism: rank r owns rows [m_lo, m_hi) of U with the
matching R rows, and rows [n_lo, n_hi) of V with the matching R columns. A
half-sweep is: Gram G = F^T F of the replicated other factor (one GEMM),
K5 ridge SPD inverse (csrc/kernels/als.hip, f64 in LDS, once — not per row),
local rows = (R_rows F) G^-1 (K5 als_solve: one pass over R_rows on the bf16 MFMA with
a hi/lo split, G^-1 applied in the epilogue), all_gather of the factor rows. The
RMSE never materialises U V^T: on the GPU the K5 residual kernel squares each f32
residual in one pass over R; on the CPU the f64 closed form ||R||^2 - 2<U, RV> +
<U^T U, V^T V> (one scalar all-reduce either way).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from dalgo.ops import _ext
from dalgo.ops import random as drandom
from dalgo.parallel import comm
from dalgo.parallel.sharding import even_slices
from dalgo.utils.obs import NULL_PHASE


@dataclass
class ALSConfig:
    m: int = 100            # users   (matrix_decomposition.py:13)
    n: int = 500            # items   (:14)
    k: int = 10             # rank    (:15)
    lam: float = 0.01       # (:12)
    n_iterations: int = 5   # (:16)
    n_workers: int = 4      # n_slices (:17)
    seed: int = 7


def rows_solve(R: torch.Tensor, F: torch.Tensor, Ginv: torch.Tensor) -> torch.Tensor:
    """(R F) Ginv for every row of R at once: K5 on the GPU (csrc/kernels/als.hip:
    R streamed once through a 3-product bf16 split MFMA GEMM, K-split partials reduced
    and multiplied by Ginv in the epilogue); torch GEMMs on the CPU."""
    if not R.is_cuda:
        return (R @ F) @ Ginv
    if R.stride(1) != 1 or R.stride(0) % 4 or R.data_ptr() % 16:
        R = _aligned_rows(R)
    out = torch.empty((R.shape[0], F.shape[1]), dtype=torch.float32, device=R.device)
    _ext.ops().als_solve(R, F.contiguous(), Ginv.contiguous(), out)
    return out


def gram(F: torch.Tensor) -> torch.Tensor:
    """F^T F: K5 split-n Gram kernel on the GPU (the library GEMM runs this skinny shape
    on a handful of workgroups), torch on the CPU."""
    if not F.is_cuda:
        return F.T @ F
    k = F.shape[1]
    G = torch.empty((k, k), dtype=torch.float32, device=F.device)
    _ext.ops().als_gram(F.contiguous(), G)
    return G


def _aligned_rows(R: torch.Tensor) -> torch.Tensor:
    ld = (R.shape[1] + 3) // 4 * 4
    buf = torch.zeros((R.shape[0], ld), dtype=R.dtype, device=R.device)
    buf[:, : R.shape[1]] = R
    return buf[:, : R.shape[1]]


def spd_inverse(G: torch.Tensor, ridge: float) -> torch.Tensor:
    """(G + ridge*I)^-1 for a small SPD G (k <= 128)."""
    out = torch.empty_like(G)
    if G.is_cuda:
        _ext.ops().spd_inverse(G.contiguous(), float(ridge), out, None)
        return out
    k = G.shape[0]
    A = G.double() + ridge * torch.eye(k, dtype=torch.float64)
    return torch.linalg.inv(A).to(G.dtype)


@dataclass
class ALSHistory:
    rmse: list = field(default_factory=list)


class ALS:
    def __init__(self, cfg: ALSConfig, rank: int = 0, world: int = 1, device="cpu",
                 dtype: torch.dtype | None = None):
        self.cfg = cfg
        dev = torch.device(device)
        self.dev = dev
        self.dtype = dtype or (torch.float32 if dev.type == "cuda" else torch.float64)
        m, n, k = cfg.m, cfg.n, cfg.k
        self.world = world
        self.rank = rank
        # synthetic rank-k R = Ut Vt^T with U(0,1) factors, plus U(0,1) initial U, V
        Ut = self._uniform(m, k, stream=11)
        Vt = self._uniform(n, k, stream=12)
        self.U = self._uniform(m, k, stream=13)
        self.V = self._uniform(n, k, stream=14)
        self.mrows = even_slices(m, world)
        self.nrows = even_slices(n, world)
        self.m_lo, self.m_hi = self.mrows[rank]
        self.n_lo, self.n_hi = self.nrows[rank]
        self.R_rows = (Ut[self.m_lo: self.m_hi] @ Vt.T).contiguous()        # [m_l, n]
        self.R_cols = (Vt[self.n_lo: self.n_hi] @ Ut.T).contiguous()        # [n_l, m] = R^T rows
        if dev.type != "cuda":   # ||R||^2 of the CPU closed-form RMSE (the GPU squares residuals)
            self.R2 = torch.tensor([float((self.R_rows.double() ** 2).sum())], dtype=torch.float64,
                                   device=dev)
            comm.all_reduce_sum(self.R2)
        self.history = ALSHistory()
        self.t = 0
        self.timer = None   # dalgo.utils.obs.PhaseTimer (None = off)
        self.bytes_gathered = 0

    def _ph(self, name: str):
        return self.timer.phase(name) if self.timer is not None else NULL_PHASE

    def _uniform(self, rows, cols, stream):
        out = torch.empty((rows, cols), dtype=torch.float32, device=self.dev)
        drandom.philox_fill_(out, D=cols, seed=self.cfg.seed, stream=stream, a=0.0, b=1.0)
        return out.to(self.dtype)

    def _gather_rows(self, local: torch.Tensor, slices, full_rows: int) -> torch.Tensor:
        counts = [b - a for a, b in slices]
        if self.world == 1:
            return local
        with self._ph("allgather"):
            out = comm.all_gather_varlen(local, counts)
        self.bytes_gathered += out.numel() * out.element_size()
        return out

    def _half(self, R_local: torch.Tensor, F: torch.Tensor, x_dim: int) -> torch.Tensor:
        with self._ph("gram+inverse"):
            G = gram(F)                                     # Gram, once per half-sweep
            Ginv = spd_inverse(G.contiguous(), self.cfg.lam * x_dim)
        with self._ph("solve"):
            return rows_solve(R_local, F, Ginv)             # all local rows at once (K5)

    def step(self):
        c = self.cfg
        U_loc = self._half(self.R_rows, self.V, x_dim=c.n)       # update(i, V, R): X_dim = n
        self.U = self._gather_rows(U_loc, self.mrows, c.m)
        V_loc = self._half(self.R_cols, self.U, x_dim=c.m)       # update(j, U, R^T): X_dim = m
        self.V = self._gather_rows(V_loc, self.nrows, c.n)
        self.t += 1

    def rmse(self) -> float:
        """sqrt(||R - U V^T||^2 / (m n)) (matrix_decomposition.py:19-21). GPU: the K5 residual
        kernel squares every f32 residual of this rank's rows in one pass over R (no m x n
        product is stored, and nothing cancels); CPU: the f64 closed form
        ||R||^2 - 2<U, RV> + <U^T U, V^T V>. One scalar all-reduce."""
        U_l = self.U[self.m_lo: self.m_hi]
        if self.R_rows.is_cuda:
            R = self.R_rows
            if R.stride(1) != 1 or R.stride(0) % 4 or R.data_ptr() % 16:
                R = _aligned_rows(R)
            part = torch.zeros(1, dtype=torch.float64, device=self.dev)
            _ext.ops().als_residual(R, U_l.float().contiguous(), self.V.float().contiguous(), part)
            comm.all_reduce_sum(part)
            sse = float(part.item())
        else:
            RV = self.R_rows.double() @ self.V.double()
            Ud, Vd = U_l.double(), self.V.double()
            part = torch.stack([-2.0 * (Ud * RV).sum(), ((Ud.T @ Ud) * (Vd.T @ Vd)).sum()])
            comm.all_reduce_sum(part)
            sse = float(self.R2.item() + part.sum().item())
        return math.sqrt(max(sse, 0.0) / (self.cfg.m * self.cfg.n))

    def state_dict(self) -> dict:
        """Replicated state: both factors (full, after the half-sweep gathers)."""
        return {"t": self.t, "U": self.U.cpu(), "V": self.V.cpu(), "rmse": list(self.history.rmse)}

    def load_state_dict(self, sd: dict):
        self.t = int(sd["t"])
        self.U = sd["U"].to(self.dev, self.dtype)
        self.V = sd["V"].to(self.dev, self.dtype)
        self.history.rmse = list(sd.get("rmse", []))

    def fit(self, n_iterations: int | None = None, callback=None):
        n = self.cfg.n_iterations if n_iterations is None else n_iterations
        for _ in range(n):
            self.step()
            with self._ph("rmse"):
                self.history.rmse.append(self.rmse())
            if callback:
                callback(self)
        return self.history
