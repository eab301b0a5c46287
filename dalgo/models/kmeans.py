"""Distributed Lloyd k-means (machine_learning/k-means.py).

Reference loop (k-means.py:53-71): ``takeSample(False, k, 42)`` initial centres,
then ``n_iterations`` x [map(closest_center) -> reduceByKey((sum, count)) ->
collect means -> replace non-empty centres]. ``convergeDist`` (:16) is declared
but never used; here ``tol`` optionally stops when the max squared centre shift
drops below it (off by default = reference behaviour).

SPMD version per iteration, every rank on its HBM-resident row shard:
  K2 assign (MFMA distance GEMM + argmin)  ->  K3 per-cluster sums/counts (full pass,
  or -- GPU, from the second iteration on, while at most DALGO_KM_INC_MAX (25 %) of
  the rank's points changed cluster -- the incremental form: only the moved points
  are subtracted from their old and added to their new cluster's f64 local sums, their
  signed entries counting-sorted by cluster and summed in runs (kmeans.hip
  km_dsegsum_kernel; per-row f64 atomics below 16k moved rows, kmeans_inc.hip))  ->
  ONE all_reduce of the fused f32 bucket [sums k x DP || counts as 2 x k exact f32
  words]  ->  fused update.
The reduceByKey shuffle + driver collect become one RCCL all-reduce whose size is
independent of N (520 KB at k=1024, d=128). Counts travel as (cnt mod 2^b,
cnt >> b) f32 pairs with b = 24 - ceil(log2 W) (21 at 8 ranks): every partial sum
of the low words stays below 2^24, so the f32 reduction is exact.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from dalgo.ops import kmeans as K
from dalgo.parallel import comm
from dalgo.utils.obs import NULL_PHASE


@dataclass
class KMeansConfig:
    k: int = 2                 # k-means.py:15
    n_iterations: int = 5      # k-means.py:18
    n_workers: int = 2         # n_slices (k-means.py:17)
    init: str = "sample"       # "sample": k distinct random rows (takeSample) | "given"
    seed: int = 42             # takeSample(False, k, 42)
    tol: float | None = None   # convergeDist-style early stop (reference ignores it)


@dataclass
class KMeansHistory:
    sse: list = field(default_factory=list)
    shift: list = field(default_factory=list)


def sample_rows(n_global: int, k: int, seed: int) -> np.ndarray:
    """k distinct global row ids (the takeSample stand-in; deterministic)."""
    if k > n_global:
        raise ValueError("k larger than the number of points")
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n_global, size=k, replace=False))


class KMeans:
    def __init__(self, cfg: KMeansConfig, X_local: torch.Tensor, row_offset: int, n_global: int,
                 init_centers: torch.Tensor | None = None):
        self.cfg = cfg
        self.X = K.prepare_points(X_local)
        self.dev = self.X.device
        self.row_offset = row_offset
        self.n_global = n_global
        self.d = self.X.shape[1]
        self.DP = K.kmeans_dp(self.d)
        k = cfg.k
        if init_centers is None:
            init_centers = self._sample_init()
        # centre-stationary K2 (kmeans_cs.hip) when it applies: centres padded to
        # 256 / 512 / 1024, fixed point statistics computed once
        kp = K.cs_kpad(k, self.d, self.X.dtype, self.dev)
        self.pstats = K.point_stats(self.X) if kp is not None else None
        self.cen = K.make_centers(init_centers.float(), self.X.dtype, self.dev, kpad=kp)
        self.assign = torch.zeros(self.X.shape[0], dtype=torch.int32, device=self.dev)
        # [S (k x DP) || count lo (k) || count hi (k)]: one all-reduce per iteration
        self.bucket = torch.zeros(k * self.DP + 2 * k, dtype=torch.float32, device=self.dev)
        self.S = self.bucket[: k * self.DP].view(k, self.DP)
        self._cnt_pair = self.bucket[k * self.DP:].view(2, k)
        self.cnt = torch.zeros(k, dtype=torch.int64, device=self.dev)
        self.bytes_allreduced = 0
        self.sse = torch.zeros(1, dtype=torch.float64, device=self.dev)
        self.shift2 = torch.zeros(1, dtype=torch.float32, device=self.dev)
        self.history = KMeansHistory()
        self.t = 0
        self.timer = None   # dalgo.utils.obs.PhaseTimer (None = off)
        # incremental K3 state (GPU): f64 local sums / counts of the last iteration and
        # its assignment (self.assign); None until a full pass has produced them
        # the sorted incremental pass costs ~0.1 ms per million signed entries (2 per moved
        # row) against ~5.5 ms for the full K3 + |x|^2 sums at 100M rows: break-even ~25 %
        self.inc_max = float(os.environ.get("DALGO_KM_INC_MAX", "0.25"))
        self._S64 = None
        self.changed_history: list = []
        # bound-filtered Lloyd (GPU, bf16, pipelined K2; DALGO_KM_BOUNDS=0 turns it off):
        # exact -- a point is skipped only when the triangle inequality proves its centre
        # is still the strictly closest one (see _step_bounds)
        self.bounds = (self.dev.type == "cuda" and self.X.dtype == torch.bfloat16
                       and self.DP in (64, 128) and self.pstats is None
                       and K.assign_variant(self.X) == 52 and self.inc_max > 0
                       and k <= 2048   # per-cluster |x|^2 sums: one LDS histogram
                       and os.environ.get("DALGO_KM_BOUNDS", "1") != "0")
        self._u = None
        self.active_history: list = []

    def _ph(self, name: str):
        return self.timer.phase(name) if self.timer is not None else NULL_PHASE

    def _sample_init(self) -> torch.Tensor:
        ids = sample_rows(self.n_global, self.cfg.k, self.cfg.seed)
        C = torch.zeros((self.cfg.k, self.d), dtype=torch.float32, device=self.dev)
        lo, hi = self.row_offset, self.row_offset + self.X.shape[0]
        mine = np.nonzero((ids >= lo) & (ids < hi))[0]
        if len(mine):
            rows = torch.from_numpy(ids[mine] - lo).to(self.dev)
            C[torch.from_numpy(mine).to(self.dev)] = self.X[rows].float()
        comm.all_reduce_sum(C)
        return C

    def _bounds_state(self):
        n, k = self.X.shape[0], self.cfg.k
        st = K.point_stats(self.X, keep_xh=True)
        self._xh = st.xh
        self._tol = 2.0 * st.M * 2.0 ** -14          # slack of a kernel distance
        self._u = torch.empty(n, dtype=torch.float32, device=self.dev)
        self._l = torch.empty(n, dtype=torch.float32, device=self.dev)
        self._mind = torch.empty(n, dtype=torch.float32, device=self.dev)
        self._mind2 = torch.empty(n, dtype=torch.float32, device=self.dev)
        self._a_prev = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)
        self._idx = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)
        self._changed = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)
        self._n_active = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._n_changed = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._Q = torch.zeros(k, dtype=torch.float64, device=self.dev)
        self._S64 = torch.empty(self.S.shape, dtype=torch.float64, device=self.dev)
        self._cnt64 = torch.empty_like(self.cnt)
        self._cq_prev = torch.empty((k, self.DP), dtype=self.cen.Cq.dtype, device=self.dev)
        # first use of the f64 cdist / reductions loads their library kernels (~0.2 s):
        # pay it here, in the full first pass, not in the first filtered iteration
        K.centre_bounds(self.cen.Cq, self.cen.Cq, k)

    def _step_bounds(self):
        """One Lloyd iteration with Hamerly's bounds (exact).

        u[x] >= |x - c_a| and l[x] <= |x - c| for every other centre c, both for the
        centres of the previous assignment (K2 writes the best and the second-best
        distance). Centre a moved by delta[a] since and no centre by more than maxd, so
        if u + delta[a] < max(s[a], l - maxd) (s[a] = half the distance from c_a to its
        nearest other centre) c_a is still strictly the closest centre and x keeps it
        without computing any distance (Hamerly, "Making k-means even faster", 2010).
        The other points go through K2 (row indirection, variant 52, top-2 epilogue) and
        the moved ones through the incremental K3. The SSE comes from the identity
        sum_c (Q_c - 2 c.S_c + n_c |c|^2) with Q_c the per-cluster sum of |x|^2,
        maintained with the sums."""
        n, k, d = self.X.shape[0], self.cfg.k, self.d
        if self._u is None:
            if not hasattr(self, "_xh") or self._S64 is None:
                self._bounds_state()
            with self._ph("assign"):
                K.assign_rows(self.X, self.cen, None, n, self.assign, self._mind, self._mind2)
            with self._ph("accumulate"):
                K.accumulate(self.X, self.assign, k, self.DP, self.S, self.cnt)
                self._S64.copy_(self.S)
                self._cnt64.copy_(self.cnt)
                K.cluster_sq_sums(self.assign, self._xh, k, self._Q)
            torch.sqrt(self._mind.clamp_min(0) + self._tol, out=self._u)
            torch.sqrt((self._mind2 - self._tol).clamp_min(0), out=self._l)
            self.active_history.append(n)
        else:
            delta, s = K.centre_bounds(self.cen.Cq, self._cq_prev, k)
            maxd = delta.max().reshape(1)
            with self._ph("filter"):
                m = K.filter_rows(self.assign, self._u, self._l, delta, s, maxd, self._a_prev,
                                  self._idx, self._n_active)
            self.active_history.append(m)
            with self._ph("assign"):
                K.assign_rows(self.X, self.cen, self._idx, m, self.assign, self._mind, self._mind2)
            with self._ph("post"):
                moved = K.post_rows(self._idx, m, self.assign, self._a_prev, self._mind,
                                    self._mind2, self._tol, self._u, self._l, self._changed,
                                    self._n_changed)
            self.changed_history.append(moved)
            if moved <= self.inc_max * n:
                with self._ph("accumulate_incremental"):
                    K.move_rows(self.X, self.DP, self._changed, moved, self.assign, self._a_prev,
                                self._S64, self._cnt64, self._xh, self._Q)
                    self.S.copy_(self._S64)
                    self.cnt.copy_(self._cnt64)
            else:
                with self._ph("accumulate"):
                    K.accumulate(self.X, self.assign, k, self.DP, self.S, self.cnt)
                    self._S64.copy_(self.S)
                    self._cnt64.copy_(self.cnt)
                    K.cluster_sq_sums(self.assign, self._xh, k, self._Q)
        # local SSE on the (rounded) centres of this assignment
        Cd = self.cen.Cq[:k, :d].double()
        Sd = self._S64[:, :d]
        sse = self._Q - 2.0 * (Cd * Sd).sum(dim=1) + self._cnt64.double() * (Cd * Cd).sum(dim=1)
        self.sse.copy_(sse.sum().clamp_min(0).reshape(1))
        self._cq_prev.copy_(self.cen.Cq[:k])

    def step(self):
        self.sse.zero_()
        self.S.zero_()
        self.cnt.zero_()
        self.shift2.zero_()
        if self.bounds:
            self._step_bounds()
            self._reduce_and_update()
            return
        inc = self._S64 is not None and self.inc_max > 0
        a_out = self._a_new if inc else self.assign
        with self._ph("assign"):
            K.assign(self.X, self.cen, out=a_out, sse=self.sse, stats=self.pstats)
        moved = None
        if inc:
            with self._ph("diff"):
                moved = K.changed_rows(a_out, self.assign, self._changed, self._n_changed)
            self.changed_history.append(moved)
            if moved > self.inc_max * self.X.shape[0]:
                inc = False
        if inc:
            with self._ph("accumulate_incremental"):
                K.move_rows(self.X, self.DP, self._changed, moved, a_out, self.assign,
                            self._S64, self._cnt64)
                self.S.copy_(self._S64)
                self.cnt.copy_(self._cnt64)
        else:
            with self._ph("accumulate"):
                K.accumulate(self.X, a_out, self.cfg.k, self.DP, self.S, self.cnt)
            self._keep_local_sums()
        if a_out is not self.assign:
            self.assign, self._a_new = a_out, self.assign
        self._reduce_and_update()

    def _reduce_and_update(self):
        W = comm.world_size()
        if W > 1:
            with self._ph("allreduce"):
                b = 24 - max(1, (W - 1).bit_length())
                self._cnt_pair[0].copy_(self.cnt & ((1 << b) - 1))
                self._cnt_pair[1].copy_(self.cnt >> b)
                comm.all_reduce_sum(self.bucket)
                torch.add(self._cnt_pair[0].to(torch.int64),
                          self._cnt_pair[1].to(torch.int64) << b, out=self.cnt)
            self.bytes_allreduced += self.bucket.numel() * 4
        with self._ph("update"):
            K.update(self.cen, self.S, self.cnt, self.shift2)
        self.t += 1

    def _keep_local_sums(self):
        """After a full K3 pass: remember the local sums for the incremental form."""
        if not (self.X.is_cuda and self.inc_max > 0):
            return
        if self._S64 is None:
            n = self.X.shape[0]
            self._S64 = torch.empty(self.S.shape, dtype=torch.float64, device=self.dev)
            self._cnt64 = torch.empty_like(self.cnt)
            self._a_new = torch.empty_like(self.assign)
            self._changed = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)
            self._n_changed = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._S64.copy_(self.S)
        self._cnt64.copy_(self.cnt)

    def fit(self, n_iterations: int | None = None, track: bool = True):
        n = self.cfg.n_iterations if n_iterations is None else n_iterations
        for _ in range(n):
            self.step()
            if track or self.cfg.tol is not None:
                sse = self.sse.clone()
                comm.all_reduce_sum(sse)
                self.history.sse.append(float(sse.item()))
                self.history.shift.append(float(self.shift2.item()))
                if self.cfg.tol is not None and self.history.shift[-1] < self.cfg.tol:
                    break
        comm.check_device_errors("end of k-means fit")
        return self.history

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        Xp = K.prepare_points(X)
        st = K.point_stats(Xp) if self.pstats is not None else None
        return K.assign(Xp, self.cen, stats=st)

    @property
    def centers(self) -> torch.Tensor:
        return self.cen.C

    def state_dict(self) -> dict:
        return {"t": self.t, "centers": self.cen.C.detach().to("cpu", copy=True), "sse": list(self.history.sse),
                "shift": list(self.history.shift)}

    def load_state_dict(self, sd: dict):
        self._S64 = None          # the next iteration runs the full K3 pass
        self._u = None            # ... and the full assignment (bounds rebuilt)
        self.t = int(sd["t"])
        self.cen.C.copy_(sd["centers"].to(self.dev))
        K.refresh(self.cen)
        self.history.sse = list(sd.get("sse", []))
        self.history.shift = list(sd.get("shift", []))
