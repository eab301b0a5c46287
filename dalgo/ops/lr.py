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

# Launch geometry of the row-streaming kernels (tuned on MI355X: bench/lr_kernel_sweep.py,
# profiles/round1-3). One launch shape remains (csrc/kernels/lr_grad.hip launch_shape).
TARGET_BLOCKS = int(os.environ.get("DALGO_LR_BLOCKS", "256"))   # workgroups per launch
                           # (split over segments): one per CU
# (192 for large steps measured 1.2-1.5 % faster in an isolated fused-step loop at 5M-10M
# rows, but not in bench.py's one-kernel step, and 7 % slower in the persistent form:
# profiles/round4/r4_10/, r4_11/ -- kept at 256)
FINE_GROUPS = 8            # switch in-block work claims from 256-row groups to 64-row
                           # quarters once fewer than this many groups are unclaimed
UNIT_SHIFT = 6             # sampled steps: work units of 2^6 rows (the final, fine claims
                           # take one unit: how closely a block's 8 waves finish together)
RPB_ALIGN = int(os.environ.get("DALGO_LR_RPB_ALIGN", "256"))
                           # granularity (rows) of each block's static range (4-row ranges
                           # measured equal: profiles/final/README.md)
# persistent launches: this fraction of the rows (the top of the range) is left out of the
# blocks' static ranges and claimed across blocks in 2^POOL_SHIFT-row chunks (the blocks that
# finish their own rows early take them: the last block no longer sets the step time).
# 10M x 1024 bf16 on one MI355X: 0.3321 ms/step without, 0.3193 / 0.3168 / 0.3153 / 0.3164
# with 5 / 10 / 15 / 20 % pooled (one-kernel form 0.3287 on the same box,
# profiles/round6/r6_37); 1.25M rows: flat (54.3 -> 54.4 us, r6_36)
POOL_FRAC = float(os.environ.get("DALGO_LR_POOL", "0.15"))
POOL_SHIFT = int(os.environ.get("DALGO_LR_POOL_SHIFT", "9"))   # rows per block claim: 2^9
# the same for one-step fused (one-kernel) launches: 10M x 1024 bf16, 20 steps, alternating
# runs on one box: 0.3353 -> 0.3274 ms/step with 10 % pooled (profiles/round6/r6_44)
POOL_FRAC_ONE = float(os.environ.get("DALGO_LR_POOL1", "0.1"))
# only where the blocks' static ranges are long: at 1.25M rows (the 8-GPU per-rank share)
# the pool cost 1-2 % (r6_36, r6_43)
POOL_MIN_ROWS = int(os.environ.get("DALGO_LR_POOL_MIN_ROWS", str(4_000_000)))
# DETERMINISTIC = combine per-block partials with the fixed-order two-level hand-off
# (bitwise repeatable) instead of float atomics (race-detection mode)
DETERMINISTIC = os.environ.get("DALGO_DETERMINISTIC", "0") == "1"
ATOMIC_EPILOGUE = 256      # flag bit of the kernel's atomic epilogue


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


def _grid(n_rows: int, nseg: int, target_blocks: int | None = None):
    """Blocks per segment and static rows per block (a multiple of RPB_ALIGN)."""
    per_seg = max(1, (target_blocks or TARGET_BLOCKS) // max(1, nseg))
    rpb = max(256, int(math.ceil(n_rows / per_seg / RPB_ALIGN)) * RPB_ALIGN)
    return max(1, int(math.ceil(n_rows / rpb))), rpb


@dataclass
class _Workspace:
    slab: torch.Tensor
    gslab: torch.Tensor
    cnt1: torch.Tensor
    cnt2: torch.Tensor
    ticket: torch.Tensor   # fused-tail arrival counter (re-armed by the kernel)
    epoch: torch.Tensor    # persistent launches: device step-release counter ...
    perr: torch.Tensor     # ... and its wait-timeout error word
    pool: torch.Tensor     # persistent launches: cross-block unit counters (per step parity)
    epochs: int = 0        # host mirror of `epoch` (advanced by nsteps per launch)
    pool_used: bool = False  # a pooled launch can raise perr too (bounded chunk-slot wait)


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
            epoch=torch.zeros(1, dtype=torch.int32, device=device),
            perr=torch.zeros(1, dtype=torch.int32, device=device),
            pool=torch.zeros(2, dtype=torch.int32, device=device),
        )
        _ws_cache[key] = ws
    return ws


def persistent_error() -> int:
    """Local error word of the persistent launches (non-zero: a step-release wait
    timed out, the launch ended early and the model is not trustworthy)."""
    e = 0
    for ws in _ws_cache.values():
        if ws.epochs or ws.pool_used:
            e = max(e, int(ws.perr.item()))
    return e


def persistent_used() -> bool:
    """True once a persistent launch has armed its step-release workspace."""
    return any(ws.epochs or ws.pool_used for ws in _ws_cache.values())


def reset_persistent_error():
    """Clear the error words AND re-arm every device counter a failed launch can leave
    behind: blocks that gave up on a step-release wait return without taking their
    ticket, pool chunks or hand-off counts, so a later launch would run its tail early
    (stale ticket) or skip pooled rows (stale pool counter). The step-release epoch
    restarts at 0 with its host mirror. Call after the failed launch has drained (the
    collective check synchronises) and before the next gradient launch."""
    for ws in _ws_cache.values():
        ws.perr.zero_()
        ws.ticket.zero_()
        ws.pool.zero_()
        ws.cnt1.zero_()
        ws.cnt2.zero_()
        ws.epoch.zero_()
        ws.epochs = 0


def check_persistent():
    """Local (this rank only) form of the persistent-launch check; multi-rank callers
    use the collective :func:`dalgo.parallel.comm.check_device_errors`."""
    if persistent_error() != 0:
        raise RuntimeError("persistent K1 launch: a step-release wait timed out")


def lr_grad(X: torch.Tensor, y: torch.Tensor, W: torch.Tensor, seg: torch.Tensor, *,
            D: int, has_bias: bool = True, eps: float = 0.0, seed: int = 42, step: int = 0,
            frac: float = 1.0, row_offset: int = 0, G: torch.Tensor | None = None,
            C: torch.Tensor | None = None, max_seg_rows: int | None = None,
            target_blocks: int | None = None, fine_groups: int | None = None,
            count_acc: torch.Tensor | None = None, g_is_zero: bool = False,
            deterministic: bool | None = None, tail: dict | None = None,
            step_dev: torch.Tensor | None = None, step_mul: int = 1):
    """Per-segment gradient SUM and selected-row COUNT.

    X: [n, >=D] (bf16/f32), y: [n] f32, W: [n_seg, ldw] f32 models,
    seg: int64 [n_seg+1] local row bounds (segment s uses W[s]).
    Returns (G [n_seg, ldw], C [n_seg]); G[:, D] is the bias gradient. ``count_acc``
    (f64) accumulates the local selected-row count.

    Epilogue: by default every block adds its partial sums to G/C with float
    atomics (G/C are zeroed here unless the caller passes ``g_is_zero=True``, e.g.
    after a ``sync_update(..., zero_grad=True)``); ``deterministic=True`` (or
    DALGO_DETERMINISTIC=1) uses the fixed-order two-level reduction instead, which
    is bitwise repeatable.

    Fused tail (GPU, one segment, atomic epilogue): ``tail`` = dict(mode 0 = SSGD /
    1 = GD, reg, eta, lam, reg_alpha, count_acc, xg) makes the LAST block of the
    launch all-reduce ``[G || C]`` over xGMI (``xg``: a shared XgmiAllReduce, or None
    on one rank), apply the update to ``W`` and leave G / C zeroed — a whole
    synchronous training step in one launch. ``count_acc`` then accumulates the
    GLOBAL minibatch size. ``tail["nsteps"] > 1``: one persistent launch runs that many
    steps (every block resident; the tail block releases each step's model).

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
        nst = int(tail.get("nsteps", 1)) if tail is not None else 1
        pool_lo = None
        pf = POOL_FRAC if nst > 1 else POOL_FRAC_ONE
        if nseg == 1 and pf > 0 and not det and int(max_seg_rows) >= POOL_MIN_ROWS:
            # static ranges over the rows below pool_lo (a 256-row multiple), the rest pooled
            nr = int(max_seg_rows)
            pool_lo = max(256, (int(nr * (1.0 - pf)) // 256) * 256)
            # (a block takes at most 64 chunks per step: the pool never needs more)
            if pool_lo >= nr or nr - pool_lo > 64 * (1 << POOL_SHIFT) * max(1, TARGET_BLOCKS // 2):
                pool_lo = None
        gx, rpb = _grid(max(int(max_seg_rows if pool_lo is None else pool_lo), 1), nseg, target_blocks)
        S = ((D + 2 + 63) // 64) * 64
        ws = _workspace(X.device, nseg, gx, S)
        fg = FINE_GROUPS if fine_groups is None else int(fine_groups)
        flags = ((fg & 0xff) << 16) | ((UNIT_SHIFT & 0xf) << 24)
        dev = dict(step_dev=step_dev, step_mul=int(step_mul)) if step_dev is not None else {}
        if tail is not None:
            if det or nseg != 1:
                raise ValueError("fused tail needs the atomic epilogue and one model")
            if not g_is_zero:
                G.zero_()
                C.zero_()
            xg = tail.get("xg")
            nsteps = int(tail.get("nsteps", 1))
            kw = {}
            if xg is not None:
                xg.count(nsteps)
                kw = dict(xg_bufs=xg.bufs, xg_rank=xg.rank, xg_slot=xg.slot,
                          xg_epoch=xg.epoch_dev, xg_err=xg.err, xg_timeout=xg.timeout_s)
            if nsteps > 1:
                # persistent launch: steps step .. step + nsteps - 1, one cooperative grid
                if ws.epochs + nsteps >= 1 << 31:
                    ws.epoch.zero_()
                    ws.epochs = 0
                kw.update(nsteps=nsteps, epoch=ws.epoch, epoch_base=ws.epochs, perr=ws.perr,
                          spin_s=float(tail.get("spin_s", 2.0)))
                ws.epochs += nsteps
            if pool_lo is not None:
                kw.update(pool=ws.pool, pool_lo=pool_lo, pool_shift=POOL_SHIFT, perr=ws.perr)
                ws.pool_used = True
            _ext.ops().lr_grad(X, y, W, seg, int(row_offset), int(D), bool(has_bias), float(eps),
                               int(seed), int(step), float(frac), gx, rpb, ws.slab, ws.gslab,
                               ws.cnt1, ws.cnt2, G, C, flags | ATOMIC_EPILOGUE, count_acc,
                               ticket=ws.ticket, tail_mode=int(tail.get("mode", 0)),
                               tail_reg=int(tail.get("reg", 0)), tail_eta=float(tail.get("eta", 0.0)),
                               tail_lam=float(tail.get("lam", 0.0)),
                               tail_reg_alpha=float(tail.get("reg_alpha", 0.0)),
                               tail_count_acc=tail.get("count_acc"), **kw, **dev)
            return G, C
        if not det:
            if not g_is_zero:
                G.zero_()
                C.zero_()
            flags |= ATOMIC_EPILOGUE
        if pool_lo is not None:
            # the row pool without a fused update: the last block re-arms ticket and pool
            dev.update(ticket=ws.ticket, tail_mode=2, pool=ws.pool, pool_lo=pool_lo,
                       pool_shift=POOL_SHIFT, perr=ws.perr)
            ws.pool_used = True
        _ext.ops().lr_grad(X, y, W, seg, int(row_offset), int(D), bool(has_bias), float(eps),
                           int(seed), int(step), float(frac), gx, rpb, ws.slab, ws.gslab,
                           ws.cnt1, ws.cnt2, G, C, flags, count_acc, **dev)
        return G, C
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
        _ext.ops().lr_eval(X, y, W, seg, int(D), bool(has_bias), float(eps), gx, rpb, correct, loss)
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
