"""Loader for the in-tree gfx950 extension ``dalgo/_dalgo_hip.so``.

Policy (no silent fallbacks): an op called on a GPU tensor ALWAYS runs the
native HIP kernel; if the extension is missing or fails to load, the call raises
:class:`NativeUnavailable`. The torch-CPU reference implementations exist only
for CPU tensors (the gloo test path), never as a stand-in for a GPU kernel.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# DALGO_EXT_LIB: load another build of the extension (A/B timing of two builds in one run)
_LIB = Path(os.environ.get("DALGO_EXT_LIB") or
            Path(__file__).resolve().parent.parent / "_dalgo_hip.so")
_lock = threading.Lock()
_state = {"loaded": False, "error": None}


class NativeUnavailable(RuntimeError):
    pass


def lib_path() -> Path:
    return _LIB


def load(build_if_missing: bool = True) -> bool:
    """Load the extension once; optionally build it in-tree if absent."""
    with _lock:
        if _state["loaded"]:
            return True
        try:
            if not _LIB.exists() and build_if_missing and os.environ.get("DALGO_NO_BUILD") != "1":
                from dalgo import _build
                _build.build()
            torch.ops.load_library(str(_LIB))
            _state["loaded"] = True
            _state["error"] = None
        except Exception as e:  # pragma: no cover - exercised on broken installs
            _state["error"] = e
        return _state["loaded"]


def available() -> bool:
    return load()


def ops():
    """``torch.ops.dalgo`` — raises NativeUnavailable if the extension cannot load."""
    if not load():
        raise NativeUnavailable(
            f"dalgo native extension not available ({_LIB}): {_state['error']!r}. "
            "Build it with `python -m dalgo._build`.")
    return torch.ops.dalgo


def is_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda
