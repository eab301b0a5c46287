"""Self-launch of N ranks for the bench / app entry points.

The reference fans one driver out to ``n_slices`` Spark workers
(/root/reference/optimization/ssgd.py:17,86). Here one process per GPU is the unit:
``python bench.py --gpus N`` started without a launcher re-runs itself as a
``torch.distributed.run`` CHILD process with N ranks (rendezvous on 127.0.0.1) and
exits with its code. Nothing in this module initialises the GPU
(``torch.cuda.device_count()`` does not on this ROCm build) and the child is a new
process, never an exec of the current one.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def already_a_rank() -> bool:
    return "RANK" in os.environ or "WORLD_SIZE" in os.environ


def self_launch(gpus: int, script: str, argv: list[str], device: str = "cuda",
                backend: str | None = None, tag: str = "bench") -> int | None:
    """Run ``script argv`` as N ranks; None when this process is already a rank or N==1.

    Refuses (returns 2) when RCCL would need more GPUs than are visible: a number that
    claims N GPUs must come from N devices."""
    if gpus <= 1 or already_a_rank():
        return None
    backend = backend or ("nccl" if device == "cuda" else "gloo")
    if device == "cuda" and backend == "nccl":
        import torch
        ndev = torch.cuda.device_count()
        if gpus > ndev:
            print(f"[{tag}] --gpus {gpus} but only {ndev} GPU(s) are visible: RCCL needs one "
                  f"GPU per rank; refusing to report a {gpus}-GPU number", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(script)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def check_world(gpus: int, world: int, tag: str = "bench"):
    if gpus != world:
        raise SystemExit(f"[{tag}] --gpus {gpus} but WORLD_SIZE={world}: launch N ranks "
                         f"(or let the script start them) so N GPUs are measured")
