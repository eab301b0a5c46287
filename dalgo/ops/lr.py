"""Logistic-regression ops: fused sampled gradient (K1+K7) and evaluation (K10).

GPU tensors run ``csrc/kernels/lr_grad.hip``; CPU tensors run the torch
reference below, which draws the identical Philox minibatch
(:mod:`dalgo.utils.philox`) so CPU (gloo) and GPU runs select the same rows.

Reference semantics (all in ``/root/reference``):
  * ``logistic_f`` = 1/(exp(-x.w) + 1 [+ 1e-6])  — ssgd.py:23-24, ma.py:25-26
  * ``gradient``   = -(y - sigma) * x            — ssgd.py:27-33
  * minibatch      = points.sample(False, f, 42+t) — ssgd.py:97 (here: Philox
    Bernoulli keyed by (seed, step, global row); Spark's per-partition RNG cannot
    be matched bit-for-bit)
  * accuracy       = sigma < 0.5 -> 0 else 1       — ssgd.py:107-110
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from dalgo.ops import _ext
from dalgo.utils import philox

import os

# Launch shape of the row-streaming kernels (tuned on MI355X, see profiles/):
#   LR_VARIANT      = launch-shape variant (table in csrc/kernels/lr_grad.hip)
#   TARGET_BLOCKS   = workgroups per launch (split over segments)
LR_VARIANT = int(os.environ.get("DALGO_LR_VARIANT", "8"))   # 8 waves, pipelined, nt row loads (bench sweep)
_TARGET_BLOCKS = int(os.environ.get("DALGO_LR_BLOCKS", "256"))
#   FINE_GROUPS     = switch the in-block work claims from 256-row groups to 64-row
#                     quarters once fewer than this many groups are unclaimed (0 = off)
LR_FINE_GROUPS = int(os.environ.get("DALGO_LR_FINE", "8"))
#   UNIT_SHIFT      = sampled steps: work units of 2^UNIT_SHIFT rows; the final (fine) claims
#                     take one unit, so it sets how closely a block's 8 waves finish together
LR_UNIT_SHIFT = int(os.environ.get("DALGO_LR_UNIT_SHIFT", "6"))
#   POOL_FRAC       = share of each segment's rows left to the cross-block pool that
#                     blocks claim from once their static range is done (0 = off)
LR_POOL_FRAC = float(os.environ.get("DALGO_LR_POOL", "0"))
#   RPB_ALIGN       = granularity (rows) of each block's static range. The kernel walks
#                     any 4-aligned range: 1.25M rows with 256-row ranges is 245 blocks of
#                     5120 rows (11 CUs idle), with 4-row ranges 256 x 4884. Measured equal
#                     (1.25M: 59.3/60.2 vs 59.6/59.0 us; 10M: 361.3 vs 361.4/362.9 us,
#                     profiles/final/README.md), so the profiled 256 stays the default
LR_RPB_ALIGN = max(4, int(os.environ.get("DALGO_LR_RPB_ALIGN", "256")) // 4 * 4)
#   BALANCED        = sampled one-model launches take balanced slices of the step's
#                     compacted selection (K7 on a side stream, one step ahead) instead of
#                     walking static row ranges with in-register Bernoulli draws. Opt-in:
#                     K1 itself is 2.7 us faster at 1.25M rows (46.1 vs 48.8 us, slices of
#                     equal length), but the side-stream K7 does not overlap K1 on this
#                     stack and the per-step event hand-offs cost more than that
#                     (profiles/round3/README.md, "K1 balanced slices")
LR_BALANCED = os.environ.get("DALGO_LR_LIST", "0") == "1"
#   DETERMINISTIC   = combine per-block partials with the fixed-order two-level
#                     hand-off (bitwise repeatable) instead of float atomics
DETERMINISTIC = os.environ.get("DALGO_DETERMINISTIC", "0") == "1"


def padded_cols(D: int, dtype: torch.dtype) -> int:
    """Row stride (elements) the kernels need: a multiple of 16 bytes."""
    vec = 8 if dtype == torch.bfloat16 else 4
    return ((D + vec - 1) // vec) * vec


def pad_features(X: torch.Tensor) -> torch.Tensor:
    """Return X (or a copy) whose rows are 16-B aligned with a 16-B multiple stride.

    Columns in the stride padding are never used: the kernels multiply them by
    zero weights and never write their gradient, so any view works.
    """
    vec = 8 if X.dtype == torch.bfloat16 else 4
    if X.stride(1) == 1 and X.stride(0) % vec == 0 and X.data_ptr() % 16 == 0:
        return X
    ld = padded_cols(X.shape[1], X.dtype)
    out = torch.zeros((X.shape[0], ld), dtype=X.dtype, device=X.device)
    out[:, : X.shape[1]] = X
    return out[:, : X.shape[1]]


def _grid(n_rows: int, nseg: int, target_blocks: int | None = None, pool_frac: float = 0.0):
    """Blocks per segment and static rows per block (multiple of LR_RPB_ALIGN). With pool_frac > 0
    the static ranges cover about (1 - pool_frac) of the rows; the rest is the segment's
    cross-block pool, claimed dynamically (csrc/kernels/lr_grad.hip)."""
    per_seg = max(1, (target_blocks or _TARGET_BLOCKS) // max(1, nseg))
    static_rows = n_rows * (1.0 - min(max(pool_frac, 0.0), 0.9))
    al = LR_RPB_ALIGN
    rpb = max(256, int(math.ceil(static_rows / per_seg / al)) * al)
    gx = max(1, min(per_seg, int(math.ceil(n_rows / rpb)))) if pool_frac > 0 else \
        max(1, int(math.ceil(n_rows / rpb)))
    return gx, rpb


@dataclass
class _Workspace:
    slab: torch.Tensor
    gslab: torch.Tensor
    cnt1: torch.Tensor
    cnt2: torch.Tensor
    ticket: torch.Tensor   # fused-tail arrival counter (re-armed by the kernel)
    pool: torch.Tensor     # cross-block pool claim heads, 2 parity sets x n_seg x 64 shards
    epoch: torch.Tensor    # persistent launches: device step-release counter ...
    perr: torch.Tensor     # ... and its wait-timeout error word
    launches: int = 0      # parity of the next launch = launches & 1
    epochs: int = 0        # host mirror of `epoch` (advanced by nsteps per launch)


_ws_cache: dict = {}


def _workspace(device, nseg, gx, S) -> _Workspace:
    key = (str(device), nseg, gx, S)
    ws = _ws_cache.get(key)
    if ws is None:
        ngroups = (gx + 15) // 16
        ws = _Workspace(
            slab=torch.empty((nseg * gx, S), dtype=torch.float32, device=device),
            gslab=torch.empty((nseg * ngroups, S), dtype=torch.float32, device=device),
            cnt1=torch.zeros(nseg * ngroups, dtype=torch.int32, device=device),
            cnt2=torch.zeros(nseg, dtype=torch.int32, device=device),
            ticket=torch.zeros(1, dtype=torch.int32, device=device),
            pool=torch.zeros(2 * nseg * 64, dtype=torch.int32, device=device),
            epoch=torch.zeros(1, dtype=torch.int32, device=device),
            perr=torch.zeros(1, dtype=torch.int32, device=device),
        )
        _ws_cache[key] = ws
    return ws


class _Selection:
    """Compacted per-step Bernoulli selections for balanced K1 slices (K7 off the K1 path).

    The minibatch of step t is a pure function of (seed, t, global row), so it can be
    drawn before step t's gradient: after each K1 launch the selection of step t + 1 is
    built on a side stream (lr_select: per-chunk lists, lr_select_compact: one ascending
    list + its length) and overlaps K1(t); K1(t + 1) waits for it with a stream event and
    gives every block ``k`` consecutive entries. Two parity buffers; a buffer is rebuilt
    only after the K1 that read it has finished (event). A step that was not prefetched
    (first step, a jump after a restore) is built in order on the current stream.
    ``k`` covers the mean plus two standard deviations of the binomial total, so the
    overflow claimed at run time is rare and the last blocks are the short ones."""

    def __init__(self, device, n: int, gx: int, frac: float, seed: int, row_offset: int):
        self.n, self.gx, self.frac, self.seed, self.row_offset = n, gx, frac, seed, row_offset
        self.ch = ((n + gx - 1) // gx + 3) // 4 * 4
        self.nch = (n + self.ch - 1) // self.ch
        mean = n * frac
        sd = math.sqrt(max(n * frac * (1.0 - frac), 0.0))
        self.k = max(1, int(math.ceil((mean + 2.0 * sd) / gx)))
        size = max(gx * self.k, self.nch * self.ch, n) + 64
        i32 = dict(dtype=torch.int32, device=device)
        self.chunks = [torch.empty(self.nch * self.ch, **i32) for _ in range(2)]
        self.counts = [torch.empty(self.nch, **i32) for _ in range(2)]
        self.list = [torch.zeros(size, **i32) for _ in range(2)]
        self.total = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(2)]
        self.claim = [torch.zeros(1, **i32) for _ in range(2)]
        self.ready = [None, None]      # step whose selection the buffer holds (enqueued)
        self.used = [False, False]     # read by a K1 since it was built (claim is dirty)
        self.ev_gen = [torch.cuda.Event(), torch.cuda.Event()]
        self.ev_use = [torch.cuda.Event(), torch.cuda.Event()]
        self.side = torch.cuda.Stream(device)
        # the buffers were initialised on the current stream: side-stream builds follow it
        self.side.wait_stream(torch.cuda.current_stream(device))

    def _build(self, step: int, par: int, stream):
        ops = _ext.ops()
        with torch.cuda.stream(stream):
            ops.lr_select(int(self.seed), int(step), float(self.frac), int(self.row_offset), self.n,
                          self.ch, self.chunks[par], self.counts[par])
            ops.lr_select_compact(self.chunks[par], self.counts[par], self.ch, self.list[par],
                                  self.total[par], self.claim[par])
            self.ev_gen[par].record(stream)
        self.ready[par] = step
        self.used[par] = False

    def args(self, step: int) -> dict:
        """Launch arguments of K1(step); call right before the launch."""
        cur = torch.cuda.current_stream()
        par = step & 1
        if self.ready[par] != step:
            if self.ready[par] is not None:
                cur.wait_event(self.ev_gen[par])   # a side-stream build still writing it
            self._build(step, par, cur)
        else:
            cur.wait_event(self.ev_gen[par])
            if self.used[par]:
                self.claim[par].zero_()            # the same step again: re-arm the claims
        return dict(sel_list=self.list[par], sel_total=self.total[par], sel_k=self.k,
                    sel_claim=self.claim[par])

    def launched(self, step: int):
        """After K1(step) is enqueued: prefetch step + 1 on the side stream."""
        cur = torch.cuda.current_stream()
        par = step & 1
        self.ev_use[par].record(cur)
        self.used[par] = True
        nxt, q = step + 1, (step + 1) & 1
        if self.ready[q] == nxt:
            return
        if self.used[q]:
            self.side.wait_event(self.ev_use[q])    # the K1 that read buffer q is done
        if self.ready[q] is not None:
            self.side.wait_event(self.ev_gen[q])
        self._build(nxt, q, self.side)


_sel_cache: dict = {}


def _selection(X, n, frac, seed, row_offset, det, w_prev, step_dev, var, nseg, pf, nsteps):
    """The balanced-slice pipeline of this launch, or None when it does not apply."""
    if not (LR_BALANCED and X.is_cuda and nseg == 1 and 0.0 < frac < 1.0 and not det
            and w_prev is None and step_dev is None and pf == 0 and (var & 0xff) == 8
            and nsteps <= 1 and n >= 1 and X.stride(0) * X.element_size() <= 2048):
        return None
    if torch.cuda.is_current_stream_capturing():
        return None
    sel_rows = n * frac
    gx = _TARGET_BLOCKS if sel_rows >= 32 * _TARGET_BLOCKS else max(1, int(math.ceil(sel_rows / 32)))
    key = (str(X.device), n, gx, float(frac), int(seed), int(row_offset))
    s = _sel_cache.get(key)
    if s is None:
        if len(_sel_cache) >= 8:
            torch.cuda.synchronize(X.device)   # no launch may still use a dropped buffer
            _sel_cache.clear()
        s = _sel_cache[key] = _Selection(X.device, n, gx, float(frac), int(seed), int(row_offset))
    return s


def persistent_error() -> int:
    """Local error word of the persistent launches (non-zero: a step-release wait
    timed out, the launch ended early and the model is not trustworthy)."""
    e = 0
    for ws in _ws_cache.values():
        if ws.epochs:
            e = max(e, int(ws.perr.item()))
    return e


def persistent_used() -> bool:
    """True once a persistent launch has armed its step-release workspace."""
    return any(ws.epochs for ws in _ws_cache.values())


def reset_persistent_error():
    for ws in _ws_cache.values():
        ws.perr.zero_()


def check_persistent():
    """Local (this rank only) form of the persistent-launch check; multi-rank callers
    use the collective :func:`dalgo.parallel.comm.check_device_errors`."""
    if persistent_error() != 0:
        raise RuntimeError("persistent K1 launch: a step-release wait timed out")


def lr_grad(X: torch.Tensor, y: torch.Tensor, W: torch.Tensor, seg: torch.Tensor, *,
            D: int, has_bias: bool = True, eps: float = 0.0, seed: int = 42, step: int = 0,
            frac: float = 1.0, row_offset: int = 0, G: torch.Tensor | None = None,
            C: torch.Tensor | None = None, max_seg_rows: int | None = None,
            variant: int | None = None, target_blocks: int | None = None,
            w_prev: torch.Tensor | None = None, update: dict | None = None,
            count_acc: torch.Tensor | None = None, g_is_zero: bool = False,
            deterministic: bool | None = None, tail: dict | None = None,
            pool_frac: float | None = None, step_dev: torch.Tensor | None = None,
            step_mul: int = 1):
    """Per-segment gradient SUM and selected-row COUNT.

    X: [n, >=D] (bf16/f32), y: [n] f32, W: [n_seg, ldw] f32 models,
    seg: int64 [n_seg+1] local row bounds (segment s uses W[s]).
    Returns (G [n_seg, ldw], C [n_seg]); G[:, D] is the bias gradient.

    Fused update (GPU, one segment): with ``w_prev`` given, the kernel first applies
    the previous step's update ``update`` (dict: mode 0 = SSGD / 1 = GD, reg, eta,
    lam, reg_alpha) using the CURRENT contents of G and C, writes the new model to
    ``W`` and computes the gradient at it. ``count_acc`` (f64) accumulates the local
    selected-row count.

    Epilogue: by default every block adds its partial sums to G/C with float
    atomics (G/C are zeroed here unless the caller passes ``g_is_zero=True``, e.g.
    after a ``sync_update(..., zero_grad=True)``); ``deterministic=True`` (or
    DALGO_DETERMINISTIC=1) uses the fixed-order two-level reduction instead, which
    is bitwise repeatable. The fused-update path is always deterministic.

    Fused tail (GPU, one segment, atomic epilogue): ``tail`` = dict(mode 0 = SSGD /
    1 = GD, reg, eta, lam, reg_alpha, count_acc, xg) makes the LAST block of the
    launch all-reduce ``[G || C]`` over xGMI (``xg``: a shared XgmiAllReduce, or None
    on one rank), apply the update to ``W`` and leave G / C zeroed — a whole
    synchronous training step in one launch. ``count_acc`` then accumulates the
    GLOBAL minibatch size.

    Graph replay: with ``step_dev`` (int64 [1] on the device) the sampling stream is
    ``step + step_mul * step_dev[0]``, read by the kernel at run time, so a step captured
    once in a hipGraph keeps drawing fresh minibatches on every replay.
    """
    nseg, ldw = W.shape
    if G is None:
        G = torch.zeros((nseg, ldw), dtype=W.dtype, device=W.device)
    if C is None:
        C = torch.zeros(nseg, dtype=W.dtype, device=W.device)
    if X.is_cuda:
        if max_seg_rows is None:
            if nseg == 1:
                max_seg_rows = int(X.shape[0])
            else:
                b = seg.tolist()
                max_seg_rows = max(b[i + 1] - b[i] for i in range(nseg))
        det = DETERMINISTIC if deterministic is None else bool(deterministic)
        # dynamic work placement (cross-block pool) only with the atomic epilogue: the
        # deterministic paths keep a fixed row -> block -> wave assignment
        pf = (LR_POOL_FRAC if pool_frac is None else float(pool_frac)) \
            if (not det and w_prev is None) else 0.0
        gx, rpb = _grid(max(int(max_seg_rows), 1), nseg, target_blocks, pf)
        S = ((D + 2 + 63) // 64) * 64
        ws = _workspace(X.device, nseg, gx, S)
        pool = {}
        if step_dev is not None:
            pf = 0.0     # graph replay: no host-side launch parity
            gx, rpb = _grid(max(int(max_seg_rows), 1), nseg, target_blocks, 0.0)
            ws = _workspace(X.device, nseg, gx, S)
            pool = dict(step_dev=step_dev, step_mul=int(step_mul))
        if pf > 0:
            pool = dict(pool=ws.pool, pool_parity=ws.launches & 1)
            ws.launches += 1
        u = update or {}
        var = LR_VARIANT if variant is None else int(variant)
        if not ((var >> 16) & 0xff):
            var |= (LR_FINE_GROUPS & 0xff) << 16
        if not (var >> 24):
            var |= (LR_UNIT_SHIFT & 0xf) << 24
        nsteps_ = int(tail.get("nsteps", 1)) if tail is not None else 1
        selp = _selection(X, int(max_seg_rows), float(frac), seed, row_offset, det, w_prev,
                          step_dev, var, nseg, pf, nsteps_)
        sel = {}
        if selp is not None:
            gx = selp.gx
            ws = _workspace(X.device, nseg, gx, S)
            sel = selp.args(int(step))
        if tail is not None:
            if det or w_prev is not None or nseg != 1:
                raise ValueError("fused tail needs the atomic epilogue, one model, no prologue update")
            if not g_is_zero:
                G.zero_()
                C.zero_()
            xg = tail.get("xg")
            nsteps = int(tail.get("nsteps", 1))
            kw = {}
            if xg is not None:
                kw = dict(xg_bufs=xg.bufs, xg_rank=xg.rank, xg_slot=xg.slot,
                          xg_epoch=xg.next_epoch(nsteps), xg_err=xg.err, xg_timeout=xg.timeout_s)
            if nsteps > 1:
                # persistent launch: steps step .. step + nsteps - 1, one cooperative grid
                if pool:
                    raise ValueError("persistent launch: no cross-block work pool")
                if ws.epochs + nsteps >= 1 << 31:
                    ws.epoch.zero_()
                    ws.epochs = 0
                kw.update(nsteps=nsteps, epoch=ws.epoch, epoch_base=ws.epochs, perr=ws.perr,
                          spin_s=float(tail.get("spin_s", 2.0)))
                ws.epochs += nsteps
            _ext.ops().lr_grad(X, y, W, seg, int(row_offset), int(D), bool(has_bias), float(eps),
                               int(seed), int(step), float(frac), gx, rpb, ws.slab, ws.gslab,
                               ws.cnt1, ws.cnt2, G, C, var | 256, None, 0, 0, 0.0, 0.0, 0.0,
                               count_acc, ticket=ws.ticket, tail_mode=int(tail.get("mode", 0)),
                               tail_reg=int(tail.get("reg", 0)), tail_eta=float(tail.get("eta", 0.0)),
                               tail_lam=float(tail.get("lam", 0.0)),
                               tail_reg_alpha=float(tail.get("reg_alpha", 0.0)),
                               tail_count_acc=tail.get("count_acc"), **kw, **pool, **sel)
            if selp is not None:
                selp.launched(int(step))
            return G, C
        if not det and w_prev is None:
            if not g_is_zero:
                G.zero_()
                C.zero_()
            var |= 256                     # atomic epilogue (csrc/kernels/lr_grad.hip)
        _ext.ops().lr_grad(X, y, W, seg, int(row_offset), int(D), bool(has_bias), float(eps),
                           int(seed), int(step), float(frac), gx, rpb, ws.slab, ws.gslab,
                           ws.cnt1, ws.cnt2, G, C, var,
                           w_prev, int(u.get("mode", 0)), int(u.get("reg", 0)),
                           float(u.get("eta", 0.0)), float(u.get("lam", 0.0)),
                           float(u.get("reg_alpha", 0.0)), count_acc, **pool, **sel)
        if selp is not None:
            selp.launched(int(step))
        return G, C
    if w_prev is not None:
        from dalgo.ops import update as U
        W.copy_(w_prev.view_as(W))
        U.sync_update(W, U.SSGD if update.get("mode", 0) == 0 else U.GD_SUM, G=G, C=C,
                      reg=update.get("reg", 0), eta=update.get("eta", 0.0),
                      lam=update.get("lam", 0.0), reg_alpha=update.get("reg_alpha", 0.0))
    if step_dev is not None:
        step = int(step) + int(step_mul) * int(step_dev.view(-1)[0])
    G, C = _lr_grad_cpu(X, y, W, seg, D, has_bias, eps, seed, step, frac, row_offset, G, C)
    if count_acc is not None:
        count_acc += float(C.sum())
    return G, C


def _lr_grad_cpu(X, y, W, seg, D, has_bias, eps, seed, step, frac, row_offset, G, C):
    segb = seg.tolist()
    G.zero_()
    C.zero_()
    for s in range(W.shape[0]):
        lo, hi = segb[s], segb[s + 1]
        if hi <= lo:
            continue
        mask = philox.bernoulli_mask(seed, step, np.arange(row_offset + lo, row_offset + hi), frac)
        idx = torch.from_numpy(np.nonzero(mask)[0] + lo)
        if idx.numel() == 0:
            continue
        Xs = X[idx, :D].to(W.dtype)
        w = W[s]
        z = Xs @ w[:D]
        if has_bias:
            z = z + w[D]
        sig = 1.0 / (torch.exp(-z) + 1.0 + eps)
        r = sig - y[idx].to(W.dtype)
        G[s, :D] = r @ Xs
        if has_bias:
            G[s, D] = r.sum()
        C[s] = float(idx.numel())
    return G, C


def lr_eval(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, *, D: int,
            has_bias: bool = True, eps: float = 0.0):
    """Return (correct_count, mean_logloss) of model w ([ldw] or [1, ldw]) on (X, y)."""
    W = w.reshape(1, -1)
    n = int(X.shape[0])
    if X.is_cuda:
        gx, rpb = _grid(max(n, 1), 1)
        seg = torch.tensor([0, n], dtype=torch.int64, device=X.device)
        correct = torch.zeros(1, dtype=torch.int64, device=X.device)
        loss = torch.zeros(1, dtype=torch.float32, device=X.device)
        _ext.ops().lr_eval(X, y, W, seg, int(D), bool(has_bias), float(eps), gx, rpb, correct, loss,
                           LR_VARIANT)
        return correct, loss / max(n, 1)
    Xs = X[:, :D].to(W.dtype)
    z = Xs @ W[0, :D]
    if has_bias:
        z = z + W[0, D]
    with np.errstate(over="ignore"):
        sig = 1.0 / (torch.exp(-z) + 1.0 + eps)
    pred = torch.where(sig < 0.5, 0.0, 1.0).to(W.dtype)
    correct = (pred == y.to(W.dtype)).sum().reshape(1)
    sc = sig.clamp(1e-7, 1 - 1e-7)
    yy = y.to(W.dtype)
    loss = -(yy * torch.log(sc) + (1 - yy) * torch.log(1 - sc)).mean().reshape(1)
    return correct, loss
