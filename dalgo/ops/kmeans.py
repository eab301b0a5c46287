"""k-means ops: fused MFMA distance+argmin (K2), per-cluster accumulation (K3)
and the centroid update (csrc/kernels/kmeans.hip), plus torch-CPU references.

Layouts: points X [n, >=DP] (bf16 or f32, zero in columns [d, DP), rows 16-B
aligned); centres keep an f32 master ``C [k, d]`` plus the MFMA copy
``Cq [kpad, DP]`` in X's dtype and ``hn = 0.5*|Cq|^2`` (1e30 for padding rows),
with DP = d rounded up to 16/32/64/128 and kpad = k rounded up to 32.
"""
from __future__ import annotations

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


_scratch: dict = {}


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


def assign(X: torch.Tensor, cen: Centers, out: torch.Tensor | None = None,
           mind: torch.Tensor | None = None, sse: torch.Tensor | None = None):
    """Nearest-centre ids (int32, ties -> lowest id), squared distances, SSE.

    GPU: K2 (csrc/kernels/kmeans.hip; the pipelined MFMA form for bf16 with d > 32,
    the generic form otherwise). CPU: exact f64 scores on the rounded centres."""
    n = X.shape[0]
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=X.device)
    if X.is_cuda:
        if sse is not None and sse.numel() == 1:
            # blocks spread their SSE partials over 256 slots (one f64 address hit by
            # every block serialises ~2 ms of atomics at 100M points), summed here
            slots = _sse_slots(X.device)
            _ext.ops().kmeans_assign(X, cen.Cq, cen.hn, out, mind, slots)
            sse += slots.sum()
        else:
            _ext.ops().kmeans_assign(X, cen.Cq, cen.hn, out, mind, sse)
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
               cnt: torch.Tensor):
    """S[c, :] += sum of rows assigned to c (f32, [k, DP]); cnt[c] += count (int64).

    GPU: counting sort by cluster + per-segment register sums (one atomic d-vector per
    2048 rows; csrc/kernels/kmeans.hip kmeans_accumulate_sorted)."""
    if X.is_cuda:
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
                 n_changed: torch.Tensor) -> None:
    """Row ids whose cluster changed -> changed[:m], m -> n_changed (device; no sync)."""
    n_changed.zero_()
    _ext.ops().kmeans_diff(a_new, a_old, changed, n_changed)


class MoveWorkspace:
    """Workspace of the incremental K3 for up to ``cap`` moved rows (2 * cap signed
    entries). Sized once for the worst case (cap = every local row) so the moved-row
    count can stay on the device: the kernels derive their geometry from it."""

    def __init__(self, device, cap: int, k: int):
        self.cap = max(1, int(cap))
        n2 = 2 * self.cap
        bmax = max(1, min(4096, (n2 + CHUNK_ROWS - 1) // CHUNK_ROWS))
        i32 = dict(dtype=torch.int32, device=device)
        self.perm = torch.empty(n2, **i32)
        self.ec = torch.empty(n2, **i32)
        self.er = torch.empty(n2, **i32)
        self.block_counts = torch.empty(bmax * k, **i32)
        self.cluster_start = torch.empty(k + 1, dtype=torch.int64, device=device)
        self.seg_start = torch.empty(k + 1, dtype=torch.int64, device=device)


def move_rows(X: torch.Tensor, DP: int, changed: torch.Tensor, m_dev: torch.Tensor,
              a_new: torch.Tensor, a_old: torch.Tensor, S64: torch.Tensor, cnt: torch.Tensor,
              ws: MoveWorkspace, xh: torch.Tensor | None = None, Q: torch.Tensor | None = None,
              cnew: torch.Tensor | None = None, cold: torch.Tensor | None = None):
    """Incremental K3: S64[a_new[r]] += x_r, S64[a_old[r]] -= x_r (f64), counts likewise
    (and Q, the per-cluster sum of |x|^2 = 2 xh, when given), for the rows r in
    changed[:*m_dev] (device count, <= ws.cap). The 2m signed entries are counting-sorted
    by cluster and every wave adds a run of <= SEG_ROWS of them in f64 registers:
    ~(2m / SEG_ROWS + k) d-vector atomics. cnew / cold: the moved rows' clusters aligned
    with ``changed`` (the filtered K2 writes them): read in order instead of gathered."""
    _ext.ops().kmeans_move_sorted(X, int(DP), changed, ws.cap, a_new, a_old, S64, cnt, xh, Q,
                                  SEG_ROWS, ws.block_counts, ws.cluster_start, ws.seg_start,
                                  ws.perm, ws.ec, ws.er, m_dev, CHUNK_ROWS, cnew, cold)


# ------------------------------------------------------------------ bound-filtered Lloyd
def centre_bounds(Cq_now: torch.Tensor, Cq_prev: torch.Tensor, k: int, d: int,
                  delta: torch.Tensor | None = None, s: torch.Tensor | None = None):
    """(delta, s) for the bound filter, on the ROUNDED centres the assign kernel uses:
    delta[c] = |c_now - c_prev| rounded up, s[c] = half the distance from c to its
    nearest other centre rounded down (f64, then f32 with a relative margin). GPU: one
    launch (kmeans_inc.hip km_centre_bounds_kernel)."""
    if delta is None:
        delta = torch.empty(k, dtype=torch.float32, device=Cq_now.device)
    if s is None:
        s = torch.empty(k, dtype=torch.float32, device=Cq_now.device)
    if Cq_now.is_cuda:
        _ext.ops().kmeans_centre_bounds(Cq_now, Cq_prev, int(k), int(d), delta, s)
        return delta, s
    a = Cq_now[:k, :d].double()
    b = Cq_prev[:k, :d].double()
    delta.copy_(((a - b).norm(dim=1) * (1 + 1e-6) + 1e-6).float())
    dd = torch.cdist(a, a)
    dd.fill_diagonal_(float("inf"))
    s.copy_((0.5 * dd.min(dim=1).values * (1 - 1e-6)).float() if k > 1
            else torch.full((k,), float("inf")))
    return delta, s


def filter_rows(assign: torch.Tensor, ul: torch.Tensor, delta: torch.Tensor, s: torch.Tensor, a_prev: torch.Tensor | None, idx: torch.Tensor,
                n_active: torch.Tensor, acl: torch.Tensor | None = None) -> None:
    """Rows that may change cluster -> idx[:m] (their cluster -> a_prev[row] when given,
    and -> acl[:m] in list order when given), m -> n_active (device; no sync). The
    largest centre shift is reduced from delta in the kernel. ``ul`` [n, 2]: the Hamerly
    bounds (u, l) per row (updated in place for the rows that are skipped)."""
    n_active.zero_()
    _ext.ops().kmeans_filter(assign, ul, delta, s, a_prev, idx, n_active, acl)


# ------------------------------------------------- candidate-pruned K2 (filtered iterations)
CAND_TILE = 256          # rows per K2 block tile (4 waves x 2 point tiles x 32)
CAND16_TILE = 384        # ... of the 16x16x32 candidate form (4 waves x 6 groups x 16)


def cand16() -> bool:
    """The candidate-pruned K2 on the 16x16x32 tiling (kmeans_assign16_kernel CND: tiles of
    CAND16_TILE rows, plain or drift-compacted neighbour lists) instead of the 32x32x16
    pipelined form (DALGO_KM_CAND16=0). 100M x 128, k = 1024, same active rows: iterations
    3-5 of the overlapping-blob job 18.8 / 11.1 / 9.6 -> 16.8 / 10.0 / 8.8 ms, job 95.6 ->
    92.0 ms; separated 75.7 -> 73.8 ms (profiles/round6/r6_53)."""
    import os
    return os.environ.get("DALGO_KM_CAND16", "1") == "1"


class CandWorkspace:
    """Buffers of the candidate-pruned filtered iteration for n rows, k clusters (kpad
    padded, <= 1024): per-centre neighbour lists (nd / nb / hnb, k * kpad each), the
    cluster-sorted active rows and the tile table."""

    def __init__(self, device, n: int, k: int, kpad: int, DP: int, drift: bool = False,
                 tile: int = CAND_TILE):
        i32 = dict(dtype=torch.int32, device=device)
        i64 = dict(dtype=torch.int64, device=device)
        f32 = dict(dtype=torch.float32, device=device)
        n = max(1, int(n))
        self.k, self.kpad = int(k), int(kpad)
        self.tile = int(tile)                            # rows per tile (<=)
        self.nd = torch.empty(k * kpad, **f32)
        self.nb = torch.empty(k * kpad, **i32)
        self.hnb = torch.empty(k * kpad, **f32)
        # drift-aware lists: every entry's distance to the list's centre (aligned with nb)
        # and its centre's shift since the last iteration
        self.ndb = torch.empty(k * kpad, **f32) if drift else None
        self.dnb = torch.empty(k * kpad, **f32) if drift else None
        # cap of the drift threshold (device): the DRIFT_QUANTILE of this iteration's shifts
        self.tau_cap = torch.full((1,), float("inf"), **f32) if drift else None
        self.acl = torch.empty(n, **i32)
        self.rows = torch.empty(n, **i32)
        bmax = max(1, (n + CHUNK_ROWS - 1) // CHUNK_ROWS)
        self.nkeys = self.k                              # sort keys: the clusters
        self.block_counts = torch.empty(bmax * self.nkeys, **i32)
        self.cstart = torch.empty(self.nkeys + 1, **i64)
        self.seg_start = torch.empty(self.nkeys + 1, **i64)
        tiles = (n + self.tile - 1) // self.tile + self.nkeys
        self.tiles = torch.empty(tiles * 4, **i32)      # (cluster, first, end, -) per tile
        self.n_tiles = torch.zeros(1, **i64)

    def cand(self):
        c = [self.tiles, self.n_tiles, self.hnb, self.nb, self.nd]
        return c + [self.ndb, self.dnb, self.tau_cap] if self.ndb is not None else c


def centre_nbrs(cen: Centers, Cq_prev: torch.Tensor, delta: torch.Tensor, s: torch.Tensor,
                ws: CandWorkspace):
    """delta / s as centre_bounds, plus every centre's neighbour lists for the pruned K2
    (one launch, kmeans_inc.hip km_centre_nbrs_kernel)."""
    _ext.ops().kmeans_centre_nbrs(cen.Cq, Cq_prev, cen.hn, ws.k, cen.d, delta, s, ws.nd, ws.nb,
                                  ws.hnb, ws.ndb, ws.dnb)
    if ws.tau_cap is not None:
        # only centres slower than this quantile of the shifts are dropped: a dropped centre
        # costs the rows its shift of lower bound, which the next filter pays
        q = drift_quantile()
        if q < 1.0:
            kq = max(1, min(ws.k, int(round(q * ws.k))))
            torch.kthvalue(delta[: ws.k], kq, out=(ws.tau_cap.view(()), torch.empty((), dtype=torch.int64,
                                                                                     device=delta.device)))
        else:
            ws.tau_cap.fill_(float("inf"))


def drift_quantile() -> float:
    """Quantile of the centre shifts that caps the drift-pruning threshold
    (DALGO_KM_DRIFT_Q, default DRIFT_QUANTILE; >= 1: no cap)."""
    import os
    return float(os.environ.get("DALGO_KM_DRIFT_Q", DRIFT_QUANTILE))


# (profiles/round6/r6_6 - r6_8: 0.5 / 0.75 / 0.9 / none measured; 0.9 best over both data sets)
DRIFT_QUANTILE = 0.9


def drift_ball() -> bool:
    """Drift-aware lists: also drop the fast centres outside the Exponion ball
    (DALGO_KM_DRIFT_BALL, default on; off streams every fast centre: 94 -> 106 ms on
    overlapping blobs, profiles/round6/r6_7)."""
    import os
    return os.environ.get("DALGO_KM_DRIFT_BALL", "1") == "1"


def sort_active(idx: torch.Tensor, n_active: torch.Tensor, ws: CandWorkspace):
    """The active rows idx[:*n_active] (clusters in ws.acl) sorted by cluster -> ws.rows,
    cluster runs -> ws.cstart, tiles of CAND_TILE rows of one cluster -> ws.tiles /
    n_tiles (4 launches, device counts only)."""
    _ext.ops().kmeans_sort_active(ws.acl, idx, n_active, ws.nkeys, CHUNK_ROWS, ws.block_counts,
                                  ws.cstart, ws.seg_start, ws.rows, ws.tile, ws.tiles,
                                  ws.n_tiles)


def assign_rows(X: torch.Tensor, cen: Centers, idx: torch.Tensor | None, m: int,
                assign: torch.Tensor, mind: torch.Tensor | None = None,
                mind2: torch.Tensor | None = None, xh: torch.Tensor | None = None,
                xmax: torch.Tensor | None = None, post: dict | None = None,
                cand: CandWorkspace | None = None, extend: bool = True):
    """K2 (pipelined form) over the rows idx[:m] (all rows when idx is None).

    Full pass: assign / mind (and the second-best distance mind2, a lower bound, when
    given) written at those rows; xh / xmax: also 0.5|x|^2 per row and its maximum
    (float bits). ``post`` = dict(m_dev, a_prev, tol, ul, changed, n_changed): the
    filtered-iteration form -- the row count is m_dev (device; m its upper bound) and
    the epilogue writes the Hamerly bounds ul[row] = (u, l) (rounded outward, tol on the
    device) and appends the rows whose cluster differs from the previous one (a_prev[row],
    else post["acl"][p] -- the filter's list order -- else assign[row]) to changed (count
    in n_changed, which the caller zeroes): no host sync, no separate bound pass. In this
    form assign must hold the previous clusters: only the changed rows are written. On
    DP = 128 it runs the dense 16x16x32 top-2 K2 (kmeans_assign16_kernel, BND form).
    ``cand`` (with post; idx = cand.rows, the active rows sorted by cluster): the
    candidate-pruned form -- a tile of cluster a streams only the chunks of a's
    neighbour list within 2 max(ua) of c_a (ua = the tile's distances to c_a, computed in
    the tile prologue and rounded up); the pruned centres enter the new lower bound as
    nd_first - ua. ``extend``: where that bound would be looser than a point's second
    best, the tile streams more chunks (tight l for the next filter). A drift-aware
    workspace (``CandWorkspace(drift=True)``) also drops, past the first chunk, every
    centre whose shift is below min over the tile rows of (l - ua): such a centre is
    farther than c_a from every tile point (l bounds the distances to the previous
    centres); the kept entries are compacted in the tile prologue, the dropped ones bound
    the new l by l - (their largest shift), and no extension chunks are streamed."""
    if post is None:
        _ext.ops().kmeans_assign_idx(X, cen.Cq, cen.hn, idx, int(m), assign, [], mind, mind2, xh,
                                     xmax)
        return
    _ext.ops().kmeans_assign_idx(X, cen.Cq, cen.hn, idx, int(m), assign,
                                 cand.cand() if cand is not None else [], None, None, None, None,
                                 post["m_dev"], post.get("a_prev"), post["tol"], post["ul"],
                                 post["changed"], post["n_changed"],
                                 post.get("chg_new"), post.get("chg_old"),
                                 int(bool(extend)) | (2 if cand is not None and cand.tile == CAND16_TILE else 0),
                                 post.get("acl"))


def bounds_init(mind: torch.Tensor, mind2: torch.Tensor, xmax: torch.Tensor, n: int,
                ul: torch.Tensor, tol: torch.Tensor):
    """After the full first pass: tol = 2 M 2^-14 (M from the K2 max of 0.5|x|^2), ul =
    (u, l) per row: u = sqrt(dist + tol) rounded up, l = sqrt(dist2 - tol) rounded down
    (one launch)."""
    _ext.ops().kmeans_bounds_init(mind, mind2, xmax, int(n), ul, tol)


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
