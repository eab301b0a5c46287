"""Multi-process CPU (gloo) harness: the 'fake cluster' of SURVEY §4.1."""
import os
import pickle
import socket
import tempfile

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch
    torch.set_num_threads(1)
    from dalgo.parallel import runtime
    rt = runtime.init(backend="gloo", device="cpu")
    try:
        res = fn(rt, *args)
    finally:
        runtime.shutdown()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def run_world(fn, world=2, args=()):
    """Run fn(rt, *args) on `world` gloo ranks; returns the list of per-rank results."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), fn, args, d), nprocs=world, join=True)
        out = []
        for r in range(world):
            with open(os.path.join(d, f"r{r}.pkl"), "rb") as f:
                out.append(pickle.load(f))
        return out
