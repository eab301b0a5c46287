"""k-means ops: fused MFMA distance+argmin (K2), per-cluster accumulation (K3)
and the centroid update (csrc/kernels/kmeans.hip), plus torch-CPU references.

Layouts: points X [n, >=DP] (bf16 or f32, zero in columns [d, DP), rows 16-B
aligned); centres keep an f32 master ``C [k, d]`` plus the MFMA copy
``Cq [kpad, DP]`` in X's dtype and ``hn = 0.5*|Cq|^2`` (1e30 for padding rows),
with DP = d rounded up to 16/32/64/128 and kpad = k rounded up to 32.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from dalgo.ops import _ext


def kmeans_dp(d: int) -> int:
    for dp in (16, 32, 64, 128):
        if d <= dp:
            return dp
    raise ValueError(f"k-means kernels support d <= 128 (got {d})")


def prepare_points(X: torch.Tensor) -> torch.Tensor:
    """Return X as an [n, d] view of a zero-padded [n, DP] buffer (copy if needed)."""
    n, d = X.shape
    DP = kmeans_dp(d)
    if X.stride(1) == 1 and X.stride(0) == DP and X.data_ptr() % 16 == 0:
        return X
    buf = torch.zeros((n, DP), dtype=X.dtype, device=X.device)
    buf[:, :d] = X
    return buf[:, :d]


def _full(X: torch.Tensor) -> torch.Tensor:
    """The [n, DP] padded rows behind a prepared [n, d] view."""
    DP = kmeans_dp(X.shape[1])
    return X.as_strided((X.shape[0], DP), (X.stride(0), 1))


@dataclass
class Centers:
    C: torch.Tensor      # [k, d] f32 master
    Cq: torch.Tensor     # [kpad, DP] compute copy (X dtype)
    hn: torch.Tensor     # [kpad] f32
    k: int
    d: int

    @property
    def DP(self) -> int:
        return self.Cq.shape[1]


def make_centers(C0: torch.Tensor, dtype: torch.dtype, device, kpad: int | None = None) -> Centers:
    k, d = C0.shape
    DP = kmeans_dp(d)
    if kpad is None:
        kpad = ((k + 127) // 128) * 128     # multiple of every chunk width of the assign kernel
    assert kpad >= k and kpad % 128 == 0
    C = C0.to(device=device, dtype=torch.float32).contiguous()
    Cq = torch.zeros((kpad, DP), dtype=dtype, device=device)
    hn = torch.zeros(kpad, dtype=torch.float32, device=device)
    cen = Centers(C, Cq, hn, k, d)
    refresh(cen)
    return cen


def refresh(cen: Centers):
    """Recompute Cq / hn from the master C (host-side torch; once per init)."""
    Cq = cen.Cq
    Cq.zero_()
    Cq[: cen.k, : cen.d] = cen.C.to(Cq.dtype)
    r = Cq[: cen.k].float()
    cen.hn.fill_(1e30)
    cen.hn[: cen.k] = 0.5 * (r * r).sum(dim=1)


import os

# launch variant of the assign kernel (table in csrc/kernels/kmeans.hip). -1 = per
# dtype: f32 -> 5 (8-wave blocks capped at 128 VGPRs, two blocks per CU), bf16 -> 52
# (pipelined distance-key form: 128-centre double-buffered chunks, 3 point tiles per
# wave, last-tile software-pipelined argmin: 4.20 ms vs 4.54 ms for 26 and 4.73-5.11 ms
# for the round-1 default 14 at 20M x 128 x 1024, profiles/round2/README.md; DP < 64
# falls back to 5 in the launcher)
ASSIGN_VARIANT = int(os.environ.get("DALGO_KM_VARIANT", "-1"))
RESIDENT_VARIANTS = (11, 12, 13)
_BF16_DEFAULT = 52
_scratch: dict = {}


def assign_variant(X: torch.Tensor, variant: int | None = None) -> int:
    v = ASSIGN_VARIANT if variant is None else int(variant)
    if v < 0:
        v = _BF16_DEFAULT if X.dtype == torch.bfloat16 else 5
    return v


# ------------------------------------------------------------------ centre-stationary K2
CS_VARIANT = 60
CS_KPADS = (256, 512, 1024)


def cs_kpad(k: int, d: int, dtype: torch.dtype, device, variant: int | None = None) -> int | None:
    """Centre padding for the centre-stationary K2 (kmeans_cs.hip, DALGO_KM_VARIANT=60),
    or None if it is not selected / does not apply (bf16 points on the GPU, d in (32, 128],
    k <= 1024). Opt-in: measured 23.4 ms vs 22.8 ms for the default pipelined variant 52
    at 100M x 128, k = 1024 (MFMA busy 57.7 % vs 68.1 %, profiles/round3/README.md): with
    two waves per SIMD the 128 resident centres per wave leave no VGPRs to prefetch."""
    v = ASSIGN_VARIANT if variant is None else variant
    if torch.device(device).type != "cuda" or dtype != torch.bfloat16 or v != CS_VARIANT:
        return None
    if kmeans_dp(d) not in (64, 128) or k > 1024:
        return None
    for kp in CS_KPADS:
        if k <= kp:
            return kp
    return None


@dataclass
class PointStats:
    """Fixed per point set (the points never change between Lloyd iterations)."""
    M: float                  # >= max 0.5|x|^2 (slack against MFMA rounding)
    x2sum: float              # sum |x|^2 (f64): SSE = kernel sum + x2sum
    xh: torch.Tensor | None   # 0.5|x|^2 per point (only for per-point distances)


def point_stats(X: torch.Tensor, keep_xh: bool = False, chunk: int = 1 << 22) -> PointStats:
    n = X.shape[0]
    mx, tot = 0.0, 0.0
    xh = torch.empty(n, dtype=torch.float32, device=X.device) if keep_xh else None
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        q = 0.5 * (X[s:e].float() ** 2).sum(dim=1)
        mx = max(mx, float(q.max().item())) if e > s else mx
        tot += 2.0 * float(q.double().sum().item())
        if xh is not None:
            xh[s:e] = q
    return PointStats(mx * 1.0001 + 1e-6, tot, xh)


def _sse_slots(device) -> torch.Tensor:
    """Zeroed [256] f64 slots for the assign kernels' per-block SSE partials."""
    key = ("sse", str(device))
    t = _scratch.get(key)
    if t is None:
        t = torch.zeros(256, dtype=torch.float64, device=device)
        _scratch[key] = t
    else:
        t.zero_()
    return t


def _dist_scratch(n: int, device) -> torch.Tensor:
    """Per-point distance buffer the multi-pass resident kernel carries between passes."""
    key = str(device)
    t = _scratch.get(key)
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1), dtype=torch.float32, device=device)
        _scratch[key] = t
    return t


def assign(X: torch.Tensor, cen: Centers, out: torch.Tensor | None = None,
           mind: torch.Tensor | None = None, sse: torch.Tensor | None = None,
           variant: int | None = None, stats: PointStats | None = None):
    """Nearest-centre ids (int32, ties -> lowest id), squared distances, SSE.

    ``stats`` (from :func:`point_stats`) enables the centre-stationary K2 when the
    centres are padded to 256 / 512 / 1024 (see :func:`cs_kpad`)."""
    n = X.shape[0]
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=X.device)
    if (X.is_cuda and stats is not None and cen.Cq.shape[0] in CS_KPADS
            and variant in (None, CS_VARIANT) and (mind is None or stats.xh is not None)):
        slots = _sse_slots(X.device) if sse is not None else None
        _ext.ops().kmeans_assign_cs(X, cen.Cq, cen.hn, stats.xh, float(stats.M), out, mind, slots)
        if sse is not None:
            sse += slots.sum() + stats.x2sum
        return out
    if X.is_cuda:
        v = assign_variant(X, variant)
        md = mind
        if md is None and v in RESIDENT_VARIANTS and X.dtype == torch.bfloat16:
            md = _dist_scratch(n, X.device)
        if sse is not None and sse.numel() == 1:
            # blocks spread their SSE partials over 256 slots (one f64 address hit by
            # every block serialises ~2 ms of atomics at 100M points), summed here
            slots = _sse_slots(X.device)
            _ext.ops().kmeans_assign(X, cen.Cq, cen.hn, out, md, slots, v)
            sse += slots.sum()
        else:
            _ext.ops().kmeans_assign(X, cen.Cq, cen.hn, out, md, sse, v)
        return out
    # CPU reference: exact scores on the ROUNDED centres, f64, first maximum wins
    Xf = X[:, : cen.d].double()
    Cr = cen.Cq[: cen.k, : cen.d].double()
    score = Xf @ Cr.T - 0.5 * (Cr * Cr).sum(dim=1)[None, :]
    best = torch.argmax(score, dim=1)
    out.copy_(best.to(torch.int32))
    dist = ((Xf * Xf).sum(dim=1) - 2 * score.gather(1, best[:, None])[:, 0]).clamp_min(0)
    if mind is not None:
        mind.copy_(dist.float())
    if sse is not None:
        sse += dist.sum()
    return out


_ws: dict = {}
SEG_ROWS = 2048          # rows summed in registers per wave before one atomic flush
CHUNK_ROWS = 65536       # rows per histogram / scatter block


def _sort_ws(device, n, k):
    B = max(1, min(4096, (n + CHUNK_ROWS - 1) // CHUNK_ROWS))
    key = (str(device), n, k)
    ws = _ws.get(key)
    if ws is None:
        ws = dict(block_counts=torch.empty(B * k, dtype=torch.int32, device=device),
                  cluster_start=torch.empty(k + 1, dtype=torch.int64, device=device),
                  seg_start=torch.empty(k + 1, dtype=torch.int64, device=device),
                  perm=torch.empty(max(n, 1), dtype=torch.int32, device=device))
        _ws.clear()
        _ws[key] = ws
    return ws


def accumulate(X: torch.Tensor, a: torch.Tensor, k: int, DP: int, S: torch.Tensor,
               cnt: torch.Tensor, method: str = "sorted"):
    """S[c, :] += sum of rows assigned to c (f32, [k, DP]); cnt[c] += count (int64).

    method "sorted" (default): counting sort by cluster + per-segment register
    sums (one atomic d-vector per 2048 rows). "table": range-partitioned LDS
    accumulation tables (ds_add_f32 per element) — kept for A/B at small k.
    """
    if X.is_cuda:
        if method == "table":
            _ext.ops().kmeans_accumulate(X, a, int(k), int(DP), S, cnt)
        else:
            ws = _sort_ws(X.device, X.shape[0], int(k))
            _ext.ops().kmeans_accumulate_sorted(X, a, int(k), int(DP), SEG_ROWS, ws["block_counts"],
                                                ws["cluster_start"], ws["seg_start"], ws["perm"], S, cnt)
        return S, cnt
    d = X.shape[1]
    idx = a.long()
    S.view(k, DP)[:, :d].index_add_(0, idx, X.to(S.dtype))
    cnt.index_add_(0, idx, torch.ones_like(idx, dtype=cnt.dtype))
    return S, cnt


def changed_rows(a_new: torch.Tensor, a_old: torch.Tensor, changed: torch.Tensor,
                 n_changed: torch.Tensor) -> int:
    """Row ids whose cluster changed -> changed[:m]; returns m (one host sync)."""
    n_changed.zero_()
    _ext.ops().kmeans_diff(a_new, a_old, changed, n_changed)
    return int(n_changed.item())


# moved rows from which the incremental K3 counting-sorts its signed entries by cluster
# (below: one wave per row with f64 atomics per feature, cheaper for few rows)
MOVE_SORTED_MIN = int(os.environ.get("DALGO_KM_MOVE_SORTED_MIN", "16384"))
_mws: dict = {}


def _move_ws(device, m: int, k: int):
    cap = 1 << max(16, (2 * m - 1).bit_length())
    key = (str(device), k)
    ws = _mws.get(key)
    if ws is None or ws["cap"] < cap:
        bmax = max(1, min(4096, (cap + CHUNK_ROWS - 1) // CHUNK_ROWS))
        i32 = dict(dtype=torch.int32, device=device)
        ws = dict(cap=cap, perm=torch.empty(cap, **i32), ec=torch.empty(cap, **i32),
                  er=torch.empty(cap, **i32), block_counts=torch.empty(bmax * k, **i32),
                  cluster_start=torch.empty(k + 1, dtype=torch.int64, device=device),
                  seg_start=torch.empty(k + 1, dtype=torch.int64, device=device))
        _mws[key] = ws
    return ws


def move_rows(X: torch.Tensor, DP: int, changed: torch.Tensor, m: int, a_new: torch.Tensor,
              a_old: torch.Tensor, S64: torch.Tensor, cnt: torch.Tensor,
              xh: torch.Tensor | None = None, Q: torch.Tensor | None = None):
    """Incremental K3: S64[a_new[r]] += x_r, S64[a_old[r]] -= x_r (f64), counts likewise
    (and Q, the per-cluster sum of |x|^2 = 2 xh, when given), for the m changed rows r.

    From MOVE_SORTED_MIN rows on, the 2m signed entries are counting-sorted by cluster
    (the K3 hist / scan / scatter kernels) and every wave adds a run of <= SEG_ROWS of them
    in f64 registers: ~(2m / SEG_ROWS + k) d-vector atomics instead of 2 * d per row."""
    k = S64.numel() // int(DP)
    if m >= MOVE_SORTED_MIN and k <= 2048:
        ws = _move_ws(X.device, int(m), k)
        B = max(1, min(4096, (2 * int(m) + CHUNK_ROWS - 1) // CHUNK_ROWS))
        _ext.ops().kmeans_move_sorted(X, int(DP), changed, int(m), a_new, a_old, S64, cnt, xh, Q,
                                      SEG_ROWS, ws["block_counts"][: B * k], ws["cluster_start"],
                                      ws["seg_start"], ws["perm"], ws["ec"], ws["er"])
        return
    _ext.ops().kmeans_move(X, int(DP), changed, int(m), a_new, a_old, S64, cnt, xh, Q)


# ------------------------------------------------------------------ bound-filtered Lloyd
def centre_bounds(Cq_now: torch.Tensor, Cq_prev: torch.Tensor, k: int):
    """(delta, s) for the bound filter, on the ROUNDED centres the assign kernel uses:
    delta[c] = |c_now - c_prev| rounded up, s[c] = half the distance from c to its
    nearest other centre rounded down (f64 then f32 with a relative margin)."""
    a = Cq_now[:k].double()
    b = Cq_prev[:k].double()
    delta = (a - b).norm(dim=1) * (1 + 1e-6) + 1e-6
    dd = torch.cdist(a, a)
    dd.fill_diagonal_(float("inf"))
    s = 0.5 * dd.min(dim=1).values * (1 - 1e-6)
    if k == 1:
        s = torch.full_like(s, float("inf"))
    return delta.float(), s.float()


def filter_rows(assign: torch.Tensor, u: torch.Tensor, l: torch.Tensor, delta: torch.Tensor,
                s: torch.Tensor, maxd: torch.Tensor, a_prev: torch.Tensor, idx: torch.Tensor,
                n_active: torch.Tensor) -> int:
    """Rows that may change cluster -> idx[:m] (their cluster -> a_prev); returns m."""
    n_active.zero_()
    _ext.ops().kmeans_filter(assign, u, l, delta, s, maxd, a_prev, idx, n_active)
    return int(n_active.item())


def assign_rows(X: torch.Tensor, cen: Centers, idx: torch.Tensor | None, m: int,
                assign: torch.Tensor, mind: torch.Tensor, mind2: torch.Tensor | None = None):
    """K2 (variant 52) over the rows idx[:m] (all rows when idx is None); assign / mind
    (and the second-best distance mind2, a lower bound, when given) written at those rows."""
    _ext.ops().kmeans_assign_idx(X, cen.Cq, cen.hn, idx, int(m), assign, mind, mind2)


def post_rows(idx: torch.Tensor, m: int, assign: torch.Tensor, a_prev: torch.Tensor,
              mind: torch.Tensor, mind2: torch.Tensor, tol: float, u: torch.Tensor,
              l: torch.Tensor, changed: torch.Tensor, n_changed: torch.Tensor) -> int:
    """u = sqrt(dist + tol), l = sqrt(dist2 - tol) for the re-assigned rows; rows whose
    cluster changed -> changed[:c]; returns c."""
    n_changed.zero_()
    _ext.ops().kmeans_post(idx, int(m), assign, a_prev, mind, mind2, float(tol), u, l, changed,
                           n_changed)
    return int(n_changed.item())


def cluster_sq_sums(assign: torch.Tensor, xh: torch.Tensor, k: int, Q: torch.Tensor):
    """Q[c] = sum of |x|^2 over the rows assigned to c (f64)."""
    Q.zero_()
    _ext.ops().kmeans_qsum(assign, xh, int(k), Q)


def update(cen: Centers, S: torch.Tensor, cnt: torch.Tensor, shift2: torch.Tensor | None = None):
    """c = S/n (non-empty), stale otherwise (k-means.py:70-71); refreshes Cq / hn."""
    if cen.C.is_cuda:
        _ext.ops().kmeans_update(cen.C, S, cnt, cen.Cq, cen.hn, shift2)
        return cen
    Sv = S.view(-1, cen.DP)[: cen.k, : cen.d]
    n = cnt[: cen.k].to(torch.float32).view(-1, 1)
    new = torch.where(n > 0, Sv / n.clamp_min(1), cen.C)
    if shift2 is not None:
        shift2 += ((new - cen.C) ** 2).sum()
    cen.C.copy_(new)
    refresh(cen)
    return cen
