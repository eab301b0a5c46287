"""Process-group runtime: one rank per GPU (replaces SparkSession / executors).

The reference obtains its workers from an external Spark runtime
(``SparkSession.builder.appName(..).getOrCreate()``, optimization/ssgd.py:78-81;
``spark.stop()``, ssgd.py:117). Here every rank is an SPMD process started by
``torchrun`` (``bench.py --gpus N`` starts it as a child process by itself),
bound to GPU ``LOCAL_RANK``, talking RCCL (torch backend ``"nccl"``) over xGMI;
on CPU-only hosts the same code runs on ``gloo``. A single process without any
launcher environment is a valid world of size 1 (no process group needed).

Device sharing rule: at init every rank publishes the identity of its GPU
(host, PCI domain/bus/device, UUID). When two ranks sit on the same physical
GPU (the one-GPU multi-rank rehearsals), :attr:`Runtime.shared_device` is True
on EVERY rank, and the library never builds a kernel that waits on another
process's kernel (K11 one-shot exchange, persistent / one-kernel K1 forms):
those need the peer kernels co-resident on other CUs, which one shared device
does not guarantee.
"""
from __future__ import annotations

import datetime
import os
import sys
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Runtime:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    app_name: str = "dalgo"
    # identity string of every rank's device (index = rank); "cpu" on CPU ranks
    device_ids: tuple = ()
    # True on every rank when any two ranks share one physical GPU
    shared_device: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def synchronize(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def log(self, *args, **kw):
        """print on rank 0 only (the reference prints from the driver)."""
        if self.is_main:
            print(*args, **kw, flush=True)


_RT: Runtime | None = None


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init(backend: str | None = None, *, device: str | None = None, app_name: str = "dalgo",
         timeout_s: float = 120.0) -> Runtime:
    """Initialise (idempotent) and return the process runtime.

    backend: "nccl" (RCCL, GPU), "gloo" (CPU) or None = auto (nccl when a GPU is
    requested/available, gloo otherwise). device: "cuda" | "cpu" | None = auto.
    """
    global _RT
    if _RT is not None:
        return _RT
    rank = _env_int("RANK", 0)
    world = _env_int("WORLD_SIZE", 1)
    local_rank = _env_int("LOCAL_RANK", rank)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    if device is None:
        if backend == "gloo":
            device = "cpu"
        else:
            device = "cuda" if torch.cuda.is_available() else "cpu"
    if device == "cuda":
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("device='cuda' requested but no GPU is visible")
        dev = torch.device("cuda", local_rank % ndev)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if backend is None:
        backend = "nccl" if dev.type == "cuda" else "gloo"

    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        # an RCCL collective that exceeds the process-group timeout aborts the
        # communicator and raises on the rank (non-zero exit) instead of hanging
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    ident = device_identity(dev)
    ids = (ident,)
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, ident)
        ids = tuple(gathered)
    shared = any(i != "cpu" and ids.count(i) > 1 for i in ids)
    _RT = Runtime(rank=rank, world_size=world, local_rank=local_rank, device=dev,
                  backend=backend if world > 1 else "none", app_name=app_name,
                  device_ids=ids, shared_device=shared)
    return _RT


def device_identity(dev: torch.device) -> str:
    """Host-unique identity of a physical device ("cpu" for CPU ranks): hostname plus
    PCI domain:bus:device plus UUID, so two ranks whose HIP_VISIBLE_DEVICES map
    different indices to one card still compare equal."""
    if dev.type != "cuda":
        return "cpu"
    import socket
    p = torch.cuda.get_device_properties(dev)
    pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return f"{socket.gethostname()}/{pci}/{p.uuid}"


def spin_waits_allowed() -> bool:
    """May this run launch kernels that wait on another process's kernels?

    False whenever ranks share a physical GPU, unless the opt-in rehearsal switch
    ``DALGO_ALLOW_SHARED_SPIN=1`` is set (tests marked ``gpu_shared`` only)."""
    rt = _RT
    if rt is None or not rt.shared_device:
        return True
    return os.environ.get("DALGO_ALLOW_SHARED_SPIN", "0") == "1"


def get() -> Runtime:
    return _RT if _RT is not None else init()


_watchdog = None


def arm_watchdog(seconds: float, tag: str = "dalgo") -> None:
    """Wall-clock deadline for this rank: if the process is still running after
    ``seconds``, print a rank-tagged message plus every thread's Python stack to stderr
    and exit with status 124. Turns a hang nothing else bounds (an RCCL call stuck below
    the process-group timeout, a device wait spinning on a peer that never arrives) into
    a fast, diagnosable failure. A second call re-arms; ``seconds <= 0`` disarms."""
    global _watchdog
    import threading
    if _watchdog is not None:
        _watchdog.cancel()
        _watchdog = None
    if seconds <= 0:
        return

    def fire():
        import faulthandler
        r = os.environ.get("RANK", "0")
        print(f"[{tag}] rank {r}: wall-clock deadline of {seconds:.0f} s exceeded; "
              f"stacks follow, exiting 124", file=sys.stderr, flush=True)
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(124)

    _watchdog = threading.Timer(float(seconds), fire)
    _watchdog.daemon = True
    _watchdog.start()


_beat = [0.0]
_stall = None


def heartbeat() -> None:
    """Progress beat (every collective wrapper in :mod:`dalgo.parallel.comm` calls it)."""
    import time
    _beat[0] = time.monotonic()


def arm_stall_watchdog(seconds: float, tag: str = "dalgo") -> None:
    """Progress deadline for this rank: if no :func:`heartbeat` arrives for ``seconds``
    (every collective beats, so a multi-rank job beats at least once per iteration),
    print a rank-tagged message plus every thread's Python stack and exit 124. Unlike
    :func:`arm_watchdog` it bounds a hang without bounding the job's length. A second
    call re-arms; ``seconds <= 0`` disarms."""
    global _stall
    import threading
    import time
    if _stall is not None:
        _stall.set()
        _stall = None
    if seconds <= 0:
        return
    stop = threading.Event()
    heartbeat()

    def run():
        while not stop.wait(min(1.0, seconds / 4)):
            idle = time.monotonic() - _beat[0]
            if idle > seconds:
                import faulthandler
                r = os.environ.get("RANK", "0")
                print(f"[{tag}] rank {r}: no progress for {idle:.0f} s (stall deadline "
                      f"{seconds:.0f} s); stacks follow, exiting 124", file=sys.stderr, flush=True)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                os._exit(124)

    threading.Thread(target=run, daemon=True, name="dalgo-stall-watchdog").start()
    _stall = stop


def test_hang_point(where: str) -> None:
    """Fault-injection hook of the hang tests: ``DALGO_TEST_HANG=<rank>:<where>`` makes
    that rank stop making progress here (sleeps), as a rank stuck in a kernel would."""
    spec = os.environ.get("DALGO_TEST_HANG")
    if not spec:
        return
    r, _, w = spec.partition(":")
    if r == os.environ.get("RANK", "0") and w == where:
        import time
        print(f"[dalgo] rank {r}: DALGO_TEST_HANG at {where}", file=sys.stderr, flush=True)
        while True:
            time.sleep(3600)


def shutdown():
    """Tear down the process group (``spark.stop()`` equivalent)."""
    global _RT
    failed = False
    arm_stall_watchdog(0)
    if dist.is_available() and dist.is_initialized():
        from dalgo.parallel import comm
        try:
            comm.check_device_errors("shutdown")   # collective: every rank learns it
        except comm.DeviceCollectiveError as e:
            print(f"[dalgo] rank {dist.get_rank()}: {e}", file=sys.stderr)
        except Exception as e:
            print(f"[dalgo] device error check failed: {e}", file=sys.stderr)
        failed = comm.error_seen()
        try:
            from dalgo.parallel import xgmi
            xgmi.close_shared()
        except Exception as e:
            print(f"[dalgo] xGMI buffer release failed: {e}", file=sys.stderr)
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    _RT = None
    if failed:
        # a device collective timed out at some point of the run: exit non-zero on
        # every rank even if the caller swallowed the exception
        raise SystemExit(3)


def seed_everything(seed: int):
    import random

    import numpy as np
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
