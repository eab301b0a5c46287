"""torchrun helper: K11 one-shot all-reduce vs. an exact rank-ordered f32 reference.

All ranks may share one GPU (gloo for the bootstrap, IPC-mapped exchange buffers
for the data): exercises buffer exchange, both phases, back-to-back calls with
no host sync in between, and bitwise agreement of every rank's result.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.parallel import runtime, xgmi  # noqa: E402


def vec(it, r, n):
    g = torch.Generator().manual_seed(1000003 * it + r)
    return torch.randn(n, generator=g)


def main():
    os.environ["DALGO_XGMI"] = "1"             # force K11 (no timing race)
    rt = runtime.init(backend="gloo", device="cuda", app_name="xgmi-check")
    xg = xgmi.shared(rt.device)
    assert xg is not None, "xGMI all-reduce did not come up"
    W, r = rt.world_size, rt.rank
    iters = int(os.environ.get("XG_ITERS", "600"))
    outs, refs = [], []
    for it in range(iters):
        n = (1, 7, 1025, 4096)[it % 4]
        x = vec(it, r, n).to(rt.device)
        xg.all_reduce_(x)                      # no host sync between calls
        if it % 37 == 0 or it >= iters - 4:
            ref = torch.zeros(n)
            for q in range(W):                 # same order as the kernel
                ref = ref + vec(it, q, n)
            outs.append(x)
            refs.append(ref)
    torch.cuda.synchronize()
    xg.check()
    bad = sum(int(not torch.equal(o.cpu(), e)) for o, e in zip(outs, refs))
    assert bad == 0, f"rank {r}: {bad} mismatching results"
    if r == 0:
        print(f"XGMI_OK world={W} exchanges={xg.exchanges}", flush=True)
    runtime.shutdown()


if __name__ == "__main__":
    main()
