"""Distributed Lloyd k-means (machine_learning/k-means.py).

Reference loop (k-means.py:53-71): ``takeSample(False, k, 42)`` initial centres,
then ``n_iterations`` x [map(closest_center) -> reduceByKey((sum, count)) ->
collect means -> replace non-empty centres]. ``convergeDist`` (:16) is declared
but never used; here ``tol`` optionally stops when the max squared centre shift
drops below it (off by default = reference behaviour).

SPMD version per iteration, every rank on its HBM-resident row shard:
  K2 assign (MFMA distance GEMM + argmin)  ->  K3 per-cluster sums/counts  ->  ONE
  all_reduce of the fused f32 bucket [sums k x DP || counts as 2 x k exact f32 words]
  ->  fused update.
On the GPU the first iteration is a full pass and every later one is incremental:
the sums are linear in the assignment, so only the points whose cluster changed are
subtracted from their old and added to their new cluster's f64 local sums (counting-
sorted signed entries, csrc/kernels/kmeans.hip km_dsegsum). With bf16 points (d in
(32, 128], k <= 2048) the iterations after the first are also bound-filtered (Hamerly):
only the points the triangle inequality cannot prove unchanged go through K2 (exact up
to near-ties within the kernels' distance rounding, see KMeansConfig).
Every count (active, moved rows) stays on the device -- the kernels that consume it
read it there -- so an iteration issues its launches without a host sync.
The reduceByKey shuffle + driver collect become one RCCL all-reduce whose size is
independent of N (520 KB at k=1024, d=128). Counts travel as (cnt mod 2^b,
cnt >> b) f32 pairs with b = 24 - ceil(log2 W) (21 at 8 ranks): every partial sum
of the low words stays below 2^24, so the f32 reduction is exact.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import math

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
    bound_filter: bool = True  # GPU bf16: Hamerly-filtered iterations after the first
    candidates: bool = True    # ... whose K2 tiles (one cluster each) stream only the centres
                               # near their cluster's centre (k <= 1024)
    # filtered iterations that run the dense top-2 K2 over the active rows instead of the
    # candidate-pruned one: "auto" = the iteration right after the full pass (the first
    # centre shifts are large, few chunks prune; no cluster sort either) and, decided on
    # the device, every iteration with >= DENSE_FRACTION of the rows active; "always";
    # "never"
    dense: str = "auto"
    # candidate lists also pruned by the centre shifts (Elkan's per-centre drift bound at
    # tile granularity, with the single Hamerly l per row): past the first chunk, a centre
    # whose shift since the last iteration is below min over the tile of (l - u) cannot
    # be the nearest of any tile row
    drift: bool = True
    # GPU, k <= 2048: incremental K3 (only moved rows re-summed) and the bound-filter state.
    # Costs ~24 B/row (move workspace) + ~48 B/row (bounds, candidates) of HBM on top of X
    # (bf16 d = 128: X is 256 B/row); False = plain full-pass Lloyd, no per-row state
    incremental: bool = True
    # "Exact" for the filtered paths means: a row keeps its centre only when the triangle
    # inequality proves it is still the closest, with the kernels' distance rounding
    # (distance keys drop 5 mantissa bits of 0.5|x - c|^2 + M) folded into the bounds.
    # Two K2 forms may still resolve a near-tie (distances equal within that slack,
    # 2^-13 max|x|^2) differently; tests check every difference against the slack.


@dataclass
class KMeansHistory:
    sse: list = field(default_factory=list)
    shift: list = field(default_factory=list)


# measured crossover of the two filtered K2 forms (profiles/round5/r5_14, 100M x 128,
# k = 1024): the dense form wins at 49-100 % active rows (overlapping blobs), the pruned
# one at 19-32 % (separated blobs); at ~70 % they tie
DENSE_FRACTION = 0.4
# with drift-aware candidate lists the pruned form wins at higher active fractions: 100M x
# 128, k = 1024 (profiles/round6/r6_8): overlapping blobs 100.0 -> 93.7 ms per job (pruned
# at 49-75 % active instead of dense), separated blobs 73.8 -> 74.5 ms (iteration 3 at 70 %
# active: 17.3 -> 12.5 ms, but its looser lower bounds leave 59M instead of 32M rows active
# in iteration 4: 5.9 -> 10.8 ms)
DENSE_FRACTION_DRIFT = 0.75


def _dense_fraction(drift: bool) -> float:
    import os
    v = os.environ.get("DALGO_KM_DENSE_FRACTION")
    if v is not None:
        return float(v)
    return DENSE_FRACTION_DRIFT if drift else DENSE_FRACTION


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
        self.cen = K.make_centers(init_centers.float(), self.X.dtype, self.dev)
        n = self.X.shape[0]
        self.assign = torch.zeros(n, dtype=torch.int32, device=self.dev)
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
        # incremental K3 (GPU, k within the sorted-move kernels' LDS): f64 local sums /
        # counts of the last iteration; the move workspace is sized for every local row
        # moving, so the moved count never has to reach the host
        self.incremental = self.dev.type == "cuda" and k <= 2048 and cfg.incremental
        # bound-filtered Lloyd (GPU, bf16, pipelined K2): a point is skipped only
        # when the triangle inequality proves its centre is still the strictly closest
        self.bounds = (self.incremental and cfg.bound_filter and self.X.dtype == torch.bfloat16
                       and self.DP in (64, 128))
        self._first = True                       # next iteration is the full pass
        self._hist_n = 0
        if self.incremental:
            i32 = dict(dtype=torch.int32, device=self.dev)
            self._S64 = torch.zeros(self.S.shape, dtype=torch.float64, device=self.dev)
            self._cnt64 = torch.zeros_like(self.cnt)
            self._changed = torch.empty(max(n, 1), **i32)
            self._n_changed = torch.zeros(1, dtype=torch.int64, device=self.dev)
            self._mws = K.MoveWorkspace(self.dev, n, k)
            # per-iteration device counters (read by the properties below, after the run):
            # [active rows, moved rows, 1 if the iteration was a full pass, rows of the
            # dense filtered K2]
            self._hist = torch.zeros((64, 4), dtype=torch.int64, device=self.dev)
            if self.bounds:
                self._alloc_bounds()
            else:
                self._a_new = torch.empty(n, **i32)

    def _alloc_bounds(self):
        n, k = self.X.shape[0], self.cfg.k
        f32 = dict(dtype=torch.float32, device=self.dev)
        i32 = dict(dtype=torch.int32, device=self.dev)
        self._xh = torch.empty(max(n, 1), **f32)     # 0.5 |x|^2 (written by the full pass)
        self._xmax = torch.zeros(1, **i32)            # max 0.5 |x|^2 (float bits)
        self._tol = torch.zeros(1, **f32)             # slack of a kernel distance (device)
        # Hamerly bounds (u, l) per row as one 8-byte pair: K2 writes them at scattered rows
        self._ul = torch.empty((max(n, 1), 2), **f32)
        self._mind = torch.empty(max(n, 1), **f32)
        self._mind2 = torch.empty(max(n, 1), **f32)
        self._a_prev = torch.empty(max(n, 1), **i32)
        self._idx = torch.empty(max(n, 1), **i32)
        self._n_active = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._n_cand = torch.zeros(1, dtype=torch.int64, device=self.dev)    # device K2 choice
        self._n_dense = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._just_full = False                       # last iteration was the full pass
        self._Q = torch.zeros(k, dtype=torch.float64, device=self.dev)
        self._cq_prev = torch.empty((k, self.DP), dtype=self.cen.Cq.dtype, device=self.dev)
        self._delta = torch.empty(k, **f32)
        self._s = torch.empty(k, **f32)
        self._post_args = dict(m_dev=self._n_active, a_prev=self._a_prev, tol=self._tol, ul=self._ul,
                               changed=self._changed, n_changed=self._n_changed)
        # candidate pruning (Exponion-style at tile granularity): the active rows sorted by
        # cluster, every tile's centre stream cut to a prefix of its centre's neighbour list
        # (DALGO_KM_CAND16=1: the 16x16x32 candidate form -- 384-row tiles)
        c16 = K.cand16() and self.DP == 128
        self._cand = (K.CandWorkspace(self.dev, n, k, self.cen.Cq.shape[0], self.DP,
                                      drift=self.cfg.drift,
                                      tile=K.CAND16_TILE if c16 else K.CAND_TILE)
                      if self.cfg.candidates and self.cen.Cq.shape[0] <= 1024 else None)
        if self._cand is not None:
            # the candidate K2 takes the previous cluster from its tile and writes the moved
            # rows' new / previous clusters next to them: no a_prev pass, no gathers
            self._chg_new = torch.empty(max(n, 1), **i32)
            self._chg_old = torch.empty(max(n, 1), **i32)
            self._post_args = dict(self._post_args, a_prev=None, chg_new=self._chg_new,
                                   chg_old=self._chg_old)

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

    # ------------------------------------------------------------- iteration counters
    def _record(self, col: int, src: torch.Tensor | int):
        if self._hist_n >= self._hist.shape[0]:
            self._hist = torch.cat([self._hist, torch.zeros_like(self._hist)])
        if isinstance(src, int):
            self._hist[self._hist_n, col].fill_(src)
        else:
            self._hist[self._hist_n, col].copy_(src[0])

    @property
    def active_history(self) -> list:
        """Rows re-assigned by K2 per iteration (bound filter; every row on a full pass)."""
        if not self.bounds:
            return []
        return [int(v) for v in self._hist[: self._hist_n, 0].tolist()]

    @property
    def changed_history(self) -> list:
        """Rows whose cluster changed per incremental iteration (full passes, which
        have no previous assignment to compare with, are left out)."""
        if not self.incremental:
            return []
        h = self._hist[: self._hist_n].tolist()
        return [int(r[1]) for r in h if not r[2]]

    @property
    def dense_history(self) -> list:
        """Rows re-assigned by the dense (unpruned top-2) K2 per iteration (0: full pass or
        the candidate-pruned K2)."""
        if not self.bounds:
            return []
        return [int(v) for v in self._hist[: self._hist_n, 3].tolist()]

    def clear_history(self):
        self._hist_n = 0

    # ------------------------------------------------------------------- iterations
    def _step_bounds(self):
        """One Lloyd iteration with Hamerly's bounds (exact up to near-ties).

        u[x] >= |x - c_a| and l[x] <= |x - c| for every other centre c, both for the
        centres of the previous assignment (K2 writes the best and the second-best
        distance). Centre a moved by delta[a] since and no centre by more than maxd, so
        if u + delta[a] < max(s[a], l - maxd) (s[a] = half the distance from c_a to its
        nearest other centre) c_a is still strictly the closest centre and x keeps it
        without computing any distance (Hamerly, "Making k-means even faster", 2010).
        The other points go through K2 (row indirection, top-2 epilogue that also
        updates their bounds and collects the moved rows) and the moved ones through the
        incremental K3. The SSE comes from the identity
        sum_c (Q_c - 2 c.S_c + n_c |c|^2) with Q_c the per-cluster sum of |x|^2,
        maintained with the sums. No host sync: the active / moved counts stay on the
        device."""
        n, k, d = self.X.shape[0], self.cfg.k, self.d
        if self._first:
            self._xmax.zero_()
            with self._ph("assign"):
                # full pass: also 0.5|x|^2 per row and its maximum (the distance slack).
                # With candidate pruning the plain (top-1) pass: its l = the best distance
                # (a valid lower bound of the second best) costs the next filter little --
                # the first centre shifts are large, so l - maxd rarely decides there -- and
                # the pruned iterations rebuild tight bounds
                K.assign_rows(self.X, self.cen, None, n, self.assign, self._mind,
                              None if self._cand is not None else self._mind2,
                              xh=self._xh, xmax=self._xmax)
            with self._ph("accumulate"):
                K.accumulate(self.X, self.assign, k, self.DP, self.S, self.cnt)
                self._S64.copy_(self.S)
                self._cnt64.copy_(self.cnt)
                K.cluster_sq_sums(self.assign, self._xh, k, self._Q)
            # u / l from the K2 distances, tol = 2 M 2^-14 from the K2 max of 0.5|x|^2
            K.bounds_init(self._mind, self._mind if self._cand is not None else self._mind2,
                          self._xmax, n, self._ul, self._tol)
            self._record(0, n)
            self._record(1, 0)
            self._record(2, 1)
            self._record(3, 0)
            self._first = False
            self._just_full = True
        else:
            cw = self._cand
            # K2 form: "dense" (the candidate workspace's filter outputs -- active rows in
            # row order, their clusters in acl -- no neighbour lists / cluster sort, the
            # unpruned top-2 K2), "cand" (pruned), or "device": both launched, the active
            # count on the device picks one (the other sees a zero row count)
            mode = self.cfg.dense
            if cw is None:
                form = "bounds"
            elif mode == "always" or (mode == "auto" and self._just_full):
                form = "dense"
            elif mode == "never":
                form = "cand"
            else:
                form = "device"
            with self._ph("centres"):
                if form in ("cand", "device"):
                    K.centre_nbrs(self.cen, self._cq_prev, self._delta, self._s, cw)
                else:
                    K.centre_bounds(self.cen.Cq, self._cq_prev, k, d, self._delta, self._s)
            with self._ph("filter"):
                K.filter_rows(self.assign, self._ul, self._delta, self._s,
                              self._a_prev if cw is None else None, self._idx, self._n_active,
                              cw.acl if cw is not None else None)
                n_cand, n_dense = self._n_active, self._n_active
                if form == "device":
                    # dense iff active >= DENSE_FRACTION n (no host sync)
                    on = self._n_active >= int(math.ceil(_dense_fraction(cw.ndb is not None) * n))
                    torch.mul(self._n_active, on, out=self._n_dense)
                    torch.sub(self._n_active, self._n_dense, out=self._n_cand)
                    n_cand, n_dense = self._n_cand, self._n_dense
                if form in ("cand", "device"):
                    K.sort_active(self._idx, n_cand, cw)
            self._n_changed.zero_()
            with self._ph("assign"):
                # K2 over the active rows; its epilogue updates u / l and collects the
                # rows whose cluster changed
                # no chunk extension right after the full pass: the first centre shifts
                # are so large that the next filter never decides on l (the same active
                # rows either way, profiles/round4/r4_13), so tight l there is pure cost
                if form in ("cand", "device", "bounds"):
                    # drift-aware lists: `extend` selects whether the Exponion ball also
                    # drops centres (no extension chunks in that form)
                    ext = (K.drift_ball() if cw is not None and cw.ndb is not None
                           else not self._just_full)
                    K.assign_rows(self.X, self.cen, cw.rows if cw is not None else self._idx, n,
                                  self.assign, post=dict(self._post_args, m_dev=n_cand), cand=cw,
                                  extend=ext)
                if form in ("dense", "device"):
                    K.assign_rows(self.X, self.cen, self._idx, n, self.assign,
                                  post=dict(self._post_args, m_dev=n_dense, acl=cw.acl))
            with self._ph("accumulate_incremental"):
                K.move_rows(self.X, self.DP, self._changed, self._n_changed, self.assign,
                            self._a_prev, self._S64, self._cnt64, self._mws, self._xh, self._Q,
                            *((self._chg_new, self._chg_old) if cw is not None else (None, None)))
                self.S.copy_(self._S64)
                self.cnt.copy_(self._cnt64)
            self._record(0, self._n_active)
            self._record(1, self._n_changed)
            self._record(2, 0)
            self._record(3, n_dense if form in ("dense", "device") else 0)
            self._just_full = False
        self._hist_n += 1
        # local SSE on the (rounded) centres of this assignment
        Cd = self.cen.Cq[:k, :d].double()
        Sd = self._S64[:, :d]
        sse = self._Q - 2.0 * (Cd * Sd).sum(dim=1) + self._cnt64.double() * (Cd * Cd).sum(dim=1)
        self.sse.copy_(sse.sum().clamp_min(0).reshape(1))
        self._cq_prev.copy_(self.cen.Cq[:k])

    def _step_incremental(self):
        """Full K2 pass, incremental K3 (GPU without the bound filter)."""
        k = self.cfg.k
        if self._first:
            with self._ph("assign"):
                K.assign(self.X, self.cen, out=self.assign, sse=self.sse)
            with self._ph("accumulate"):
                K.accumulate(self.X, self.assign, k, self.DP, self.S, self.cnt)
                self._S64.copy_(self.S)
                self._cnt64.copy_(self.cnt)
            self._record(1, 0)
            self._record(2, 1)
            self._first = False
        else:
            with self._ph("assign"):
                K.assign(self.X, self.cen, out=self._a_new, sse=self.sse)
            with self._ph("diff"):
                K.changed_rows(self._a_new, self.assign, self._changed, self._n_changed)
            with self._ph("accumulate_incremental"):
                K.move_rows(self.X, self.DP, self._changed, self._n_changed, self._a_new,
                            self.assign, self._S64, self._cnt64, self._mws)
                self.S.copy_(self._S64)
                self.cnt.copy_(self._cnt64)
            self.assign, self._a_new = self._a_new, self.assign
            self._record(1, self._n_changed)
            self._record(2, 0)
        self._hist_n += 1

    def step(self):
        self.sse.zero_()
        self.S.zero_()
        self.cnt.zero_()
        self.shift2.zero_()
        if self.bounds:
            self._step_bounds()
        elif self.incremental:
            self._step_incremental()
        else:
            with self._ph("assign"):
                K.assign(self.X, self.cen, out=self.assign, sse=self.sse)
            with self._ph("accumulate"):
                K.accumulate(self.X, self.assign, self.cfg.k, self.DP, self.S, self.cnt)
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
        return K.assign(K.prepare_points(X), self.cen)

    @property
    def centers(self) -> torch.Tensor:
        return self.cen.C

    def state_dict(self) -> dict:
        return {"t": self.t, "centers": self.cen.C.detach().to("cpu", copy=True), "sse": list(self.history.sse),
                "shift": list(self.history.shift)}

    def load_state_dict(self, sd: dict):
        self._first = True        # the next iteration is the full pass (sums, bounds rebuilt)
        self.t = int(sd["t"])
        self.cen.C.copy_(sd["centers"].to(self.dev))
        K.refresh(self.cen)
        self.history.sse = list(sd.get("sse", []))
        self.history.shift = list(sd.get("shift", []))
