"""Observability: EWMA-smoothed accuracy plots, JSONL metrics, phase timers, roctx.

The algorithms (ParallelSGD, KMeans, PageRank, ALS, closure, Monte Carlo) time their
phases through :class:`PhaseTimer` when a timer is attached (the apps attach one when
``--metrics-out`` is given or DALGO_ROCTX=1), and the apps write one JSONL line per
iteration with the phase split and the bytes all-reduced.

Parity with the reference's R6 layer: ``draw_acc_plot`` / ``ewma_smooth``
(optimization/ssgd.py:50-66 — EWMA alpha 0.9, raw curve at alpha 0.3, saved as
``<algo>_acc_plot.png``) and ``display_clusters`` (machine_learning/k-means.py:30-40).
Everything is rank-0 only; plotting is skipped gracefully when matplotlib is absent.
"""
from __future__ import annotations

import contextlib
import json
import os
import time

import numpy as np
import torch


def ewma_smooth(accs, alpha: float = 0.9) -> np.ndarray:
    """s[0] = a[0]; s[i] = alpha*s[i-1] + (1-alpha)*a[i]  (ssgd.py:51-58)."""
    accs = np.asarray(accs, dtype=np.float64)
    s = np.zeros_like(accs)
    for i, a in enumerate(accs):
        s[i] = a if i == 0 else alpha * s[i - 1] + (1 - alpha) * a
    return s


def draw_acc_plot(accs, path: str, title: str = "Accuracy on test dataset") -> str | None:
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        return None
    n = len(accs)
    if n == 0:
        return None
    x = np.arange(1, n + 1)
    fig = plt.figure()
    plt.plot(x, accs, color="C0", alpha=0.3)
    plt.plot(x, ewma_smooth(accs, 0.9), color="C0")
    plt.title(label=title)
    plt.xlabel("Round")
    plt.ylabel("Accuracy")
    plt.savefig(path)
    plt.close(fig)
    return path


def display_clusters(points: np.ndarray, assign: np.ndarray, k: int, path: str,
                     seed: int = 0) -> str | None:
    """Scatter each cluster in its own random colour (k-means.py:30-40), 2-D data only."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        return None
    rng = np.random.default_rng(seed)
    fig = plt.figure()
    for c in range(k):
        p = points[assign == c]
        if len(p) == 0:
            continue
        color = "#" + "".join(rng.choice(list("0123456789ABCDEF"), 6))
        plt.scatter(p[:, 0], p[:, 1], c=color)
    plt.savefig(path)
    plt.close(fig)
    return path


NULL_PHASE = contextlib.nullcontext()


class PhaseTimer:
    """Per-phase device time of each training step, without host syncs in the hot path.

    ``with timer.phase("grad"): ...`` records a HIP event pair on the current stream
    around the enqueued work (a roctx range around the host side when DALGO_ROCTX=1)
    and files it under the current step; :meth:`take` hands the step's pairs to the
    caller (usually :meth:`MetricsSink.log`), which resolves them to milliseconds once
    the GPU has passed them (``Event.query``), never blocking the step loop. On CPU the
    phases are timed with perf_counter. Models hold ``timer = None`` by default; their
    ``_ph(name)`` then returns a shared null context (no per-step cost)."""

    def __init__(self, device: torch.device, enabled: bool = True):
        self.device = torch.device(device)
        self.enabled = enabled
        self.totals: dict[str, float] = {}
        self._cur: list = []        # (name, start, end) of the current step
        self._pending: list = []    # pairs taken by nobody yet (summary())

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        with roctx_range(name):
            if self.device.type == "cuda":
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                yield
                b.record()
                self._cur.append((name, a, b))
            else:
                t0 = time.perf_counter()
                yield
                self._cur.append((name, t0, time.perf_counter()))

    def take(self) -> list:
        """The current step's (name, start, end) records; starts the next step."""
        cur, self._cur = self._cur, []
        return cur

    @staticmethod
    def ready(recs: list) -> bool:
        return all(not isinstance(b, torch.cuda.Event) or b.query() for _, _, b in recs)

    @staticmethod
    def resolve(recs: list) -> dict[str, float]:
        """ms per phase name (sums repeated phases, e.g. MA's 5 local steps)."""
        out: dict[str, float] = {}
        for name, a, b in recs:
            ms = a.elapsed_time(b) if isinstance(a, torch.cuda.Event) else (b - a) * 1e3
            out[name] = out.get(name, 0.0) + ms
        return out

    def summary(self) -> dict[str, float]:
        """Totals over every step not taken by a sink (synchronises once)."""
        self._pending.extend(self._cur)
        self._cur = []
        if self._pending:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            for k, v in self.resolve(self._pending).items():
                self.totals[k] = self.totals.get(k, 0.0) + v
            self._pending.clear()
        return dict(self.totals)


class MetricsSink:
    """Append-only JSONL metrics (rank 0; ``None`` path = disabled).

    ``log(phases=timer.take(), **fields)``: records whose phase events the GPU has
    not passed yet are held back and written, in order, by a later ``log`` (non-
    blocking ``Event.query``) or by ``close`` (one synchronise). Each line carries
    ``phase_ms`` = {phase: device ms} next to the caller's fields (step, accuracy,
    bytes all-reduced, ...)."""

    def __init__(self, path: str | None, rank: int = 0):
        self.path = path if (path and rank == 0) else None
        self._f = open(self.path, "a") if self.path else None
        self._held: list = []

    @property
    def enabled(self) -> bool:
        return self._f is not None

    def _write(self, rec: dict, phases: list | None):
        if phases:
            rec["phase_ms"] = PhaseTimer.resolve(phases)
        self._f.write(json.dumps(rec, default=float) + "\n")

    def _drain(self, block: bool):
        while self._held:
            rec, ph = self._held[0]
            if not block and ph and not PhaseTimer.ready(ph):
                break
            if block and ph:
                for _, _, b in ph:
                    if isinstance(b, torch.cuda.Event):
                        b.synchronize()
            self._held.pop(0)
            self._write(rec, ph)
        self._f.flush()

    def log(self, phases: list | None = None, **kw):
        if not self._f:
            return
        kw.setdefault("ts", time.time())
        self._held.append((kw, phases))
        self._drain(block=False)

    def close(self):
        if self._f:
            self._drain(block=True)
            self._f.close()
            self._f = None


_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("DALGO_ROCTX") == "1":
            import ctypes
            # the rocprofiler-sdk roctx (what rocprofv3 --marker-trace intercepts) first,
            # the legacy roctracer library second
            for lib in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                        "libroctx64.so"):
                try:
                    _ROCTX = ctypes.CDLL(lib)
                    break
                except OSError:
                    continue
    return _ROCTX


def roctx_enabled() -> bool:
    return bool(_roctx())


@contextlib.contextmanager
def roctx_range(name: str):
    """roctx range (visible in rocprofv3 --marker-trace) when DALGO_ROCTX=1."""
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(name.encode())
        try:
            yield
        finally:
            lib.roctxRangePop()
    else:
        yield
