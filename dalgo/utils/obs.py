"""Observability: EWMA-smoothed accuracy plots, JSONL metrics, phase timers, roctx.

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


class MetricsSink:
    """Append-only JSONL metrics (rank 0). ``None`` path = disabled."""

    def __init__(self, path: str | None, rank: int = 0):
        self.path = path if (path and rank == 0) else None
        self._f = open(self.path, "a") if self.path else None

    def log(self, **kw):
        if self._f:
            kw.setdefault("ts", time.time())
            self._f.write(json.dumps(kw, default=float) + "\n")
            self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


class PhaseTimer:
    """Per-phase wall time with device events (HIP events on GPU, perf_counter on CPU)."""

    def __init__(self, device: torch.device, enabled: bool = True):
        self.device = device
        self.enabled = enabled
        self.totals: dict[str, float] = {}
        self._pending: list = []

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
                self._pending.append((name, a, b))
            else:
                t0 = time.perf_counter()
                yield
                self.totals[name] = self.totals.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def summary(self) -> dict[str, float]:
        if self._pending:
            torch.cuda.synchronize(self.device)
            for name, a, b in self._pending:
                self.totals[name] = self.totals.get(name, 0.0) + a.elapsed_time(b)
            self._pending.clear()
        return dict(self.totals)


_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("DALGO_ROCTX") == "1":
            try:
                import ctypes
                _ROCTX = ctypes.CDLL("libroctx64.so")
            except OSError:
                _ROCTX = False
    return _ROCTX


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
