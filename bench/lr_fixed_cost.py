"""Diagnostics: fixed per-launch cost of K1 at small minibatches (epilogue variants, grid sizes)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalgo.ops import lr as L  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for rows in (20_000, 1_250_000):
        X = torch.randn(rows, 1024, device=dev).to(torch.bfloat16)
        y = (torch.rand(rows, device=dev) < 0.5).float()
        W = torch.zeros(1, 1025, device=dev)
        seg = torch.tensor([0, rows], dtype=torch.int64, device=dev)
        G = torch.zeros(1, 1025, device=dev)
        C = torch.zeros(1, device=dev)
        for name, var, det in [("atomic", 6, False), ("two-level", 6, True),
                               ("no-epilogue", 6 | 512, True)]:
            for blocks in (64, 128, 256, 512):
                kw = dict(D=1024, frac=0.1, G=G, C=C, variant=var, target_blocks=blocks,
                          deterministic=det, g_is_zero=True)
                for i in range(20):
                    L.lr_grad(X, y, W, seg, step=i, **kw)
                torch.cuda.synchronize()
                n = 200
                t0 = time.perf_counter()
                for i in range(n):
                    L.lr_grad(X, y, W, seg, step=i, **kw)
                torch.cuda.synchronize()
                us = (time.perf_counter() - t0) / n * 1e6
                print(json.dumps({"rows": rows, "epilogue": name, "blocks": blocks, "us": round(us, 2)}))


if __name__ == "__main__":
    main()
