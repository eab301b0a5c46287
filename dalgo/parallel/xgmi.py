"""K11: one-shot xGMI all-reduce for latency-bound vectors (csrc/kernels/xgmi_allreduce.hip).

The SGD family all-reduces a ~4 KB ``[g || count]`` bucket every step
(treeAggregate, optimization/ssgd.py:99-103); at 8 GPUs that collective is a
sizeable part of a ~60 us step. MI355X GPUs in a node are fully connected by
point-to-point xGMI links, so instead of a ring every rank writes its vector
straight into every peer's exchange buffer (IPC-mapped, uncached), raises one
flag per peer and sums the W slots of its own buffer in rank order: one hop, all
links in parallel, bitwise-identical results on every rank.

Safety: the exchange buffers are opened collectively; a self-test checks exact
sums over back-to-back calls (both buffer phases), and the decision to use K11 is
itself all-reduced, so either every rank uses it or none does (falls back to
RCCL). The device-side wait is bounded by a wall-clock timeout that sets an error
word instead of hanging; :meth:`XgmiAllReduce.check` raises if it ever fired.

Selection (``DALGO_XGMI``): ``auto`` (default) times K11 against the process
group's all-reduce on a bucket-sized vector right after the self-test and keeps
whichever is faster (max over ranks, so all ranks agree); ``1`` forces K11 (if the
self-test passes), ``0`` disables it. ``DALGO_XGMI_TIMEOUT`` (s, default 5; capped
at 2 s when ranks share a GPU). K11 is never built when two ranks share one
physical GPU (:func:`dalgo.parallel.runtime.spin_waits_allowed`): its peer wait
would then depend on another process's kernel being co-resident on the same CUs.
"""
from __future__ import annotations

import os
import sys

import torch
import torch.distributed as dist

from dalgo.ops import _ext

MAX_RANKS = 8
SLOT_FLOATS = 4096          # largest vector (floats) handled; larger buckets use RCCL


def _default_timeout() -> float:
    from dalgo.parallel import runtime
    t = float(os.environ.get("DALGO_XGMI_TIMEOUT", "5"))
    rt = runtime._RT
    if rt is not None and rt.shared_device:
        t = min(t, 2.0)
    return t


def _agree(ok: bool, device) -> bool:
    """Collective AND of a per-rank flag."""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                        device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return int(flag.item()) == 1


class XgmiAllReduce:
    """Exchange buffers of all ranks + the K11 launch. Construction is collective and
    failure-consistent: it raises on EVERY rank if any rank could not allocate or
    map the buffers (no rank is left waiting in a collective)."""

    def __init__(self, device: torch.device, slot_floats: int = SLOT_FLOATS,
                 timeout_s: float | None = None, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > MAX_RANKS:
            raise ValueError(f"xGMI all-reduce supports at most {MAX_RANKS} ranks")
        self.device = torch.device(device)
        self.slot = int(slot_floats)
        self.timeout_s = float(timeout_s if timeout_s is not None else _default_timeout())
        self.own = 0
        self.opened = []
        self.bufs = []
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        handle, err = None, None
        try:
            ops = _ext.ops()
            self._ops = ops
            self.own = int(ops.xgmi_alloc(int(ops.xgmi_buffer_bytes(self.slot)), dev_index))
            handle = bytes(ops.xgmi_get_handle(self.own).numpy().tobytes())
        except Exception as e:
            err = e
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)   # every rank takes part
        if any(h is None for h in handles):
            self._release()
            raise RuntimeError(f"xGMI buffer allocation failed on some rank ({err!r})")
        try:
            for r in range(self.world):
                if r == self.rank:
                    self.bufs.append(self.own)
                else:
                    h = torch.frombuffer(bytearray(handles[r]), dtype=torch.uint8).clone()
                    p = int(self._ops.xgmi_open(h, dev_index))
                    self.opened.append(p)
                    self.bufs.append(p)
            ok = True
        except Exception as e:
            err, ok = e, False
        if not _agree(ok, self.device):
            self._release()
            raise RuntimeError(f"xGMI IPC mapping failed on some rank ({err!r})")
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # device-resident exchange epoch (csrc/include/dalgo/xgmi.h): the kernels read and
        # advance it themselves, so a step with an exchange can be captured in a hipGraph
        # and replayed; the host only counts the exchanges it enqueued (epoch-space guard)
        self.epoch_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.exchanges = 0

    def count(self, k: int = 1):
        """Account for k exchanges enqueued (eager calls, kernel tails, graph replays)."""
        self.exchanges += int(k)
        if self.exchanges >= (1 << 32) - 1:
            raise RuntimeError("xGMI all-reduce epoch space exhausted")

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        """In-place SUM over ranks of a contiguous f32 GPU vector (numel <= slot)."""
        self.count()
        self._ops.xgmi_allreduce(x, self.bufs, self.rank, self.slot, self.epoch_dev, self.err,
                                 self.timeout_s)
        return x

    def all_reduce_update_(self, x: torch.Tensor, W: torch.Tensor, *, mode: int, reg: int = 0,
                           eta: float = 0.0, lam: float = 0.0, reg_alpha: float = 0.0,
                           count_index: int, count_acc: torch.Tensor | None = None) -> torch.Tensor:
        """All-reduce the ``[g || count]`` bucket ``x`` and apply the SSGD (mode 0) or
        full-batch GD (mode 1) update to ``W`` in the same launch (fused K8); ``x`` is
        left ZEROED, ready for the next atomic-epilogue gradient kernel."""
        self.count()
        self._ops.xgmi_allreduce(x, self.bufs, self.rank, self.slot, self.epoch_dev, self.err,
                                 self.timeout_s, W, int(mode), int(reg), float(eta), float(lam),
                                 float(reg_alpha), int(count_index), count_acc)
        return x

    def check(self):
        """Local check of this rank's error word only; training code uses the
        collective :func:`dalgo.parallel.comm.check_device_errors` (raises on every rank)."""
        if int(self.err.item()) != 0:
            raise RuntimeError("xGMI all-reduce: a peer flag wait timed out (results invalid)")

    def _release(self):
        for p in self.opened:
            try:
                self._ops.xgmi_close(p)
            except Exception:
                pass
        self.opened = []
        if self.own:
            try:
                self._ops.xgmi_free(self.own)
            except Exception:
                pass
            self.own = 0

    def close(self):
        """Collective: every rank stops using the buffers before any is freed."""
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        self._release()


def _self_test(xg: XgmiAllReduce) -> bool:
    """K11 result == exact expected sums for a few back-to-back calls (both phases)."""
    n = 1031
    ok = True
    for it in range(4):
        base = torch.arange(n, dtype=torch.float32, device=xg.device)
        x = base * (xg.rank + 1) + it
        xg.all_reduce_(x)
        W = xg.world
        exp = base * (W * (W + 1) / 2) + it * W
        torch.cuda.synchronize(xg.device)
        ok = ok and bool(torch.equal(x, exp))
    return ok and int(xg.err.item()) == 0


_shared: dict = {}
# outcome of the start-up K11-vs-process-group race (bench JSON): None until a race ran
last_race: dict | None = None


def _race(xg: XgmiAllReduce, n: int = 1025, iters: int = 50) -> tuple[float, float]:
    """(K11, process group) seconds for ``iters`` back-to-back all-reduces, max over ranks."""
    import time
    x = torch.zeros(n, dtype=torch.float32, device=xg.device)
    out = []
    for use_k11 in (True, False):
        for _ in range(5):
            xg.all_reduce_(x) if use_k11 else dist.all_reduce(x)
        torch.cuda.synchronize(xg.device)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            xg.all_reduce_(x) if use_k11 else dist.all_reduce(x)
        torch.cuda.synchronize(xg.device)
        out.append(time.perf_counter() - t0)
    t = torch.tensor(out, dtype=torch.float64,
                     device=xg.device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1])


def shared(device: torch.device) -> XgmiAllReduce | None:
    """Process-wide K11 instance for the default group (collective on first call).

    Returns None (on every rank) if disabled, unsupported or the self-test fails.
    """
    key = str(device)
    if key in _shared:
        return _shared[key]
    inst = None
    mode = os.environ.get("DALGO_XGMI", "auto")
    from dalgo.parallel import runtime
    if mode in ("1", "auto") and not runtime.spin_waits_allowed():
        mode = "0"   # ranks share a GPU: no cross-process spin-waiting kernels (collective)
    if (mode in ("1", "auto") and dist.is_initialized()
            and 1 < dist.get_world_size() <= MAX_RANKS and torch.device(device).type == "cuda"
            and _ext.available()):
        try:
            inst = XgmiAllReduce(device, timeout_s=min(2.0, _default_timeout()))
        except Exception as e:   # consistent on every rank (collective construction)
            if dist.get_rank() == 0:
                print(f"[dalgo] xGMI all-reduce unavailable: {e}", file=sys.stderr)
            inst = None
        if inst is not None:
            try:
                ok = _self_test(inst)
            except Exception as e:
                print(f"[dalgo] rank {dist.get_rank()}: xGMI self-test error: {e}", file=sys.stderr)
                ok = False
            if _agree(ok, device):
                inst.timeout_s = _default_timeout()
                if mode == "auto":
                    t_k11, t_pg = _race(inst)
                    global last_race
                    last_race = {"k11_us": t_k11 / 50 * 1e6, "process_group_us": t_pg / 50 * 1e6,
                                 "winner": "k11" if t_k11 < t_pg else dist.get_backend()}
                    if dist.get_rank() == 0:
                        print(f"[dalgo] small all-reduce: xGMI one-shot {t_k11 / 50 * 1e6:.1f} us, "
                              f"{dist.get_backend()} {t_pg / 50 * 1e6:.1f} us -> "
                              f"{'xGMI' if t_k11 < t_pg else dist.get_backend()}", file=sys.stderr)
                    if not t_k11 < t_pg:
                        inst.close()
                        inst = None
            else:
                inst.close()
                inst = None
                if dist.get_rank() == 0:
                    print("[dalgo] xGMI self-test failed: using the process group's all-reduce",
                          file=sys.stderr)
    _shared[key] = inst
    return inst


def disable() -> None:
    """Collective: stop using K11 for the rest of the run (every later small all-reduce
    goes through the process group); the exchange buffers are released."""
    for k, inst in list(_shared.items()):
        if inst is not None:
            inst.err.zero_()
            inst.close()
        _shared[k] = None


def close_shared():
    """Release the shared instances (collective; called by runtime.shutdown)."""
    for k, inst in list(_shared.items()):
        if inst is not None:
            if int(inst.err.item()) != 0:
                print("[dalgo] warning: an xGMI all-reduce wait timed out during the run",
                      file=sys.stderr)
            inst.close()
        del _shared[k]
