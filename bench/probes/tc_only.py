"""K9 closure step alone (one variant, a few launches) for rocprofv3 PMC passes."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--variant", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from dalgo.models.transitive_closure import DenseClosure
    from dalgo.ops import _ext
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    n = a.n
    src = torch.randint(0, n, (4 * n,), device=dev, generator=g)
    dst = torch.randint(0, n, (4 * n,), device=dev, generator=g)
    tc = DenseClosure(src, dst, n, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    for _ in range(a.reps):
        _ext.ops().tc_step(tc.A, tc.T, tc.T2, cnt, a.variant)
    torch.cuda.synchronize()
    print("ok", int(cnt.item()))


if __name__ == "__main__":
    main()
