"""Shared command-line plumbing for the reference-compatible entry scripts.

Every script keeps the reference's constants as argparse defaults and adds the
common flags below. Launch: ``python <script>.py`` (one rank) or
``torchrun --nproc-per-node N <script>.py`` (one rank per GPU, RCCL).
"""
from __future__ import annotations

import argparse

import torch

from dalgo.parallel import runtime


def common_parser(description: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto",
                    help="cuda = gfx950 HIP kernels + RCCL, cpu = torch reference + gloo")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--metrics-out", default=None, help="JSONL metrics file (rank 0)")
    ap.add_argument("--quiet", action="store_true", help="suppress per-iteration lines")
    ap.add_argument("--no-plot", action="store_true")
    ap.add_argument("--pg-timeout-s", type=float, default=120.0,
                    help="process-group timeout (default 120 s): a collective stuck longer raises on "
                         "the rank; raise it for runs where one rank does long work (I/O, data "
                         "generation) while its peers already wait in a collective")
    ap.add_argument("--stall-timeout-s", type=float, default=300.0,
                    help="multi-rank runs (default 300 s): a rank with no progress beat for this "
                         "long prints its stacks and exits 124 (0 = off). Collectives, data "
                         "generation chunks and checkpoint writes beat")
    ap.add_argument("--deadline-s", type=float, default=0.0,
                    help="wall-clock deadline of the whole run, exit 124 past it (0 = off)")
    return ap


def add_ckpt_args(ap: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """--ckpt-dir / --ckpt-every / --resume (the reference has none)."""
    ap.add_argument("--ckpt-dir", default=None, help="checkpoint directory")
    ap.add_argument("--ckpt-every", type=int, default=0,
                    help="checkpoint every K iterations (0: only at the end)")
    ap.add_argument("--resume", action="store_true", help="continue from --ckpt-dir")
    return ap


def init_from_args(a, app_name: str) -> runtime.Runtime:
    dev = None if a.device == "auto" else a.device
    if dev is None and a.backend == "gloo":
        dev = "cpu"
    timeout = getattr(a, "pg_timeout_s", 120.0)
    if getattr(a, "deadline_s", 0.0) > 0:
        runtime.arm_watchdog(a.deadline_s, tag=app_name)
    rt = runtime.init(backend=a.backend, device=dev, app_name=app_name, timeout_s=timeout)
    if rt.distributed and getattr(a, "stall_timeout_s", 0.0) > 0:
        runtime.arm_stall_watchdog(a.stall_timeout_s, tag=app_name)
    return rt


def default_dtype(rt: runtime.Runtime, want: str | None = None) -> torch.dtype:
    if want == "bf16":
        return torch.bfloat16
    if want == "f32":
        return torch.float32
    if want == "f64":
        return torch.float64
    return torch.float32 if rt.device.type == "cuda" else torch.float64
