"""Collectives (replace the reference's Spark data-movement primitives).

Reference call site -> collective here:
  * ``sc.broadcast(w)`` every iteration (ssgd.py:95)      -> nothing (w is replicated
    SPMD); :func:`broadcast` once at init
  * ``treeAggregate`` of (sum g, count) (ssgd.py:99-103)  -> :func:`all_reduce_sum` of
    one fused ``[g || count]`` buffer (one latency-bound RCCL call per step)
  * ``reduceByKey`` + ``collect`` (k-means.py:62-67)      -> all_reduce of the fused
    ``[k*d sums || k counts]`` table
  * ``reduceByKey`` of PageRank contributions (pagerank.py:57) -> :func:`all_gather_into`
    of destination-partitioned rank slices (half the bytes of an all-reduce)
  * ``collect`` of ALS factor rows (matrix_decomposition.py:52-64) -> all_gather
  * ``count`` / ``reduce(add)`` (pagerank.py:44, monte_carlo.py:28) -> int64 all_reduce

With world size 1 every call is a no-op / identity, so single-GPU runs pay no
communication. All calls are issued on the current stream (RCCL enqueues on
its own stream, torch inserts the event dependencies), so they can be captured
with the surrounding kernels.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from dalgo.parallel import runtime


def _active() -> bool:
    # every collective wrapper enters through here: that is the progress beat the
    # stall watchdog (runtime.arm_stall_watchdog) listens for
    runtime.heartbeat()
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world_size() -> int:
    return dist.get_world_size() if _active() else 1


def rank() -> int:
    return dist.get_rank() if _active() else 0


def _xgmi_for(t: torch.Tensor):
    """The K11 one-shot all-reduce if ``t`` is a small contiguous f32 GPU vector."""
    if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
        return None
    from dalgo.parallel import xgmi
    if t.numel() > xgmi.SLOT_FLOATS:
        return None
    return xgmi.shared(t.device)   # collective on first use; None if disabled / failed


def xgmi_instance():
    """The live K11 exchange of this process (None if none was set up)."""
    from dalgo.parallel import xgmi
    for inst in xgmi._shared.values():
        if inst is not None:
            return inst
    return None


def uses_xgmi(t: torch.Tensor) -> bool:
    """Would a synchronous all_reduce_sum of ``t`` take the K11 one-shot path?"""
    return _active() and _xgmi_for(t) is not None


def all_reduce_sum(t: torch.Tensor, async_op: bool = False):
    """In-place SUM all-reduce (identity at world size 1).

    Latency-bound vectors (f32, <= 4096 floats, on GPU) take the K11 one-shot
    xGMI path (rank-ordered sum, identical on every rank); everything else RCCL.
    """
    if not _active():
        return t
    if not async_op:
        xg = _xgmi_for(t)
        if xg is not None:
            xg.all_reduce_(t)
            return t
    work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)
    return work if async_op else t


class DeviceCollectiveError(RuntimeError):
    """A device-side collective wait (K11 peer flag, persistent step release) timed
    out on some rank: the results since the last check are not trustworthy."""


_error_seen = False


def error_seen() -> bool:
    """True once :func:`check_device_errors` has raised in this process."""
    return _error_seen


# test hook: a device error word this rank reports once (exercises the recovery paths
# on hosts without device-side waits; set via DALGO_TEST_FORCE_DEVICE_ERROR in bench.py)
_forced_error = 0


def _local_error_word() -> int:
    global _forced_error
    e, _forced_error = _forced_error, 0
    from dalgo.parallel import xgmi
    for inst in list(xgmi._shared.values()):
        if inst is not None:
            e = max(e, int(inst.err.item()))
    from dalgo.ops import lr as lr_ops
    e = max(e, lr_ops.persistent_error())
    return e


def device_waits_possible() -> bool:
    """Could any device error word be set? Only K11 exchanges and persistent launches
    wait on the device (both decided identically on every rank), plus the test hook
    (an environment variable, identical on every rank). Without them the error check
    skips its collective."""
    import os
    from dalgo.parallel import xgmi
    if any(inst is not None for inst in xgmi._shared.values()):
        return True
    from dalgo.ops import lr as lr_ops
    if lr_ops.persistent_used():
        return True
    return "DALGO_TEST_FORCE_DEVICE_ERROR" in os.environ


def check_device_errors(where: str = "") -> None:
    """Collective (EVERY rank must call it at the same point): MAX over ranks of the
    device error words (K11 bounded peer-flag waits, persistent-launch step releases).
    Raises :class:`DeviceCollectiveError` on every rank if any rank's word is set, so
    no rank is left blocked in a later collective. The reduction goes through the
    process group (never K11, whose failure it reports). A no-op (no collective, no
    host sync) while no device-side wait exists on any rank."""
    global _error_seen
    if not device_waits_possible():
        return
    e = _local_error_word()
    if _active():
        dev = runtime.get().device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([e], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        e = int(t.item())
    if e:
        _error_seen = True
        at = f" (at {where})" if where else ""
        raise DeviceCollectiveError(
            f"a device-side collective wait timed out on some rank{at}: results are invalid")


def reset_device_errors() -> None:
    """Clear this rank's device error words and the raised flag (call on every rank,
    after :func:`check_device_errors` raised everywhere and the caller has switched the
    run to paths without device-side waits, e.g. :func:`dalgo.parallel.xgmi.disable`)."""
    global _error_seen
    from dalgo.parallel import xgmi
    for inst in list(xgmi._shared.values()):
        if inst is not None:
            inst.err.zero_()
    from dalgo.ops import lr as lr_ops
    lr_ops.reset_persistent_error()
    _error_seen = False


def all_reduce_max(t: torch.Tensor):
    if _active():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def all_reduce_count(n: int | torch.Tensor, device=None) -> int:
    """Global integer count (``rdd.count()`` / ``reduce(add)`` equivalent)."""
    if isinstance(n, torch.Tensor):
        t = n.to(torch.int64).reshape(1).clone()
    else:
        dev = device or runtime.get().device
        t = torch.tensor([int(n)], dtype=torch.int64, device=dev)
    all_reduce_sum(t)
    return int(t.item())


def broadcast(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _active():
        dist.broadcast(t, src=src)
    return t


def all_gather_into(out: torch.Tensor, local: torch.Tensor) -> torch.Tensor:
    """Gather equal-sized local shards into ``out`` (concatenated along dim 0)."""
    if not _active():
        if out.data_ptr() != local.data_ptr():
            out.copy_(local.reshape(out.shape))
        return out
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


def all_gather_varlen(local: torch.Tensor, counts: list[int]) -> torch.Tensor:
    """Gather shards of different lengths along dim 0 (padded all_gather + trim)."""
    if not _active():
        return local
    m = max(counts)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((m * len(counts),) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, pad)
    parts = [out[i * m: i * m + c] for i, c in enumerate(counts)]
    return torch.cat(parts, dim=0)


def reduce_scatter_sum(out: torch.Tensor, full: torch.Tensor) -> torch.Tensor:
    if not _active():
        out.copy_(full.reshape(out.shape))
        return out
    dist.reduce_scatter_tensor(out, full.contiguous(), op=dist.ReduceOp.SUM)
    return out


class _Done:
    """Handle of a collective that already completed (``async_op`` fallbacks)."""

    def wait(self):
        return True


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_split: list[int] | None = None,
                      in_split: list[int] | None = None, async_op: bool = False):
    """Personalised exchange along dim 0 (``out_split[p]`` rows arrive from rank p,
    ``in_split[p]`` rows go to it); RCCL runs it as grouped send/recv over all peers at
    once. World size 1: a copy. ``async_op``: returns a handle whose ``wait()`` orders
    the current stream after the exchange (RCCL runs it on its own stream meanwhile)."""
    if not _active():
        if out.numel():
            out.copy_(inp.reshape(out.shape))
        return _Done() if async_op else out
    if inp.is_cuda and dist.get_backend() == "gloo":
        # gloo's all_to_all takes host tensors only (the one-GPU multi-rank rehearsal)
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host, inp.cpu(), output_split_sizes=out_split,
                               input_split_sizes=in_split)
        out.copy_(host)
        return _Done() if async_op else out
    work = dist.all_to_all_single(out, inp.contiguous(), output_split_sizes=out_split,
                                  input_split_sizes=in_split, async_op=async_op)
    return work if async_op else out


class _Group:
    """Handles of one shift of :func:`exchange_by_shift` (wait() waits all of them)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


def exchange_by_shift(out: torch.Tensor, inp: torch.Tensor, out_split: list[int],
                      in_split: list[int]) -> list:
    """The personalised exchange of :func:`all_to_all_single`, issued as W - 1 grouped
    send/recv shifts (shift k: to rank + k, from rank - k; the same order on every rank,
    so the pairs always match) that all start now. Returns [(source rank, handle)] in
    shift order: a caller can consume each peer's rows as soon as they land (handle.wait()
    orders the current stream after that shift only) instead of after the whole exchange.
    Empty directions post nothing (both sides agree: the splits are each other's)."""
    W, r = world_size(), rank()
    if W == 1 or (inp.is_cuda and dist.get_backend() == "gloo"):
        all_to_all_single(out, inp, out_split, in_split)
        return [((r - k) % W, _Done()) for k in range(1, W)]
    so = [0] * (W + 1)
    ro = [0] * (W + 1)
    for p in range(W):
        so[p + 1] = so[p] + int(in_split[p])
        ro[p + 1] = ro[p] + int(out_split[p])
    res = []
    for k in range(1, W):
        dst, src = (r + k) % W, (r - k) % W
        ops = []
        if in_split[dst] > 0:
            ops.append(dist.P2POp(dist.isend, inp[so[dst]:so[dst + 1]], dst))
        if out_split[src] > 0:
            ops.append(dist.P2POp(dist.irecv, out[ro[src]:ro[src + 1]], src))
        res.append((src, _Group(dist.batch_isend_irecv(ops) if ops else [])))
    return res


def gather_to_rank0(local: torch.Tensor, counts: list[int]) -> torch.Tensor | None:
    """``collect()``: rows of every rank concatenated on rank 0 (None elsewhere)."""
    full = all_gather_varlen(local, counts)
    return full if rank() == 0 else None


class BucketedAllReduce:
    """Flatten several tensors into one contiguous bucket and all-reduce once.

    xGMI rings are per-link latency/bandwidth bound; small per-tensor
    all-reduces (the SGD family's [g||cnt], k-means' [sums||counts]) are fused
    into one RCCL call. Tensors are views into the bucket, so kernels can write
    their outputs straight into it (no pack/unpack copies).
    """

    def __init__(self, shapes: list[tuple[int, ...]], dtype=torch.float32, device=None,
                 allow_xgmi: bool = True):
        device = device or runtime.get().device
        sizes = [int(torch.Size(s).numel()) for s in shapes]
        self.buffer = torch.zeros(sum(sizes), dtype=dtype, device=device)
        self.views = []
        off = 0
        for s, n in zip(shapes, sizes):
            self.views.append(self.buffer[off: off + n].view(s))
            off += n
        # latency-bound GPU buckets go through the K11 one-shot xGMI all-reduce
        # (collective decision: all ranks or none; RCCL otherwise)
        self.xg = _xgmi_for(self.buffer) if (allow_xgmi and _active()) else None

    def all_reduce(self, async_op: bool = False):
        if self.xg is not None:
            self.xg.all_reduce_(self.buffer)   # stream-ordered: nothing to wait for
            return None if async_op else self.buffer
        return all_reduce_sum(self.buffer, async_op=async_op)
