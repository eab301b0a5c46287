"""Latency of small device -> host reads (.cpu(), .tolist(), .item(), pinned non_blocking)
in a fresh process: first and repeated calls per size (the PageRank build's host syncs)."""
import time

import torch

dev = torch.device("cuda")
torch.zeros(1, device=dev).sum().item()
for n in (1, 8, 4096, 8192, 65536, 1 << 20):
    x = torch.arange(n, device=dev, dtype=torch.int64)
    torch.cuda.synchronize()
    row = []
    for _ in range(3):
        t = time.perf_counter()
        y = x.cpu()
        row.append((time.perf_counter() - t) * 1e3)
    t = time.perf_counter()
    z = x.tolist()
    tl = (time.perf_counter() - t) * 1e3
    h = torch.empty(n, dtype=torch.int64, pin_memory=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    h.copy_(x, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    tp = (time.perf_counter() - t) * 1e3
    print(f"n={n:8d} int64: .cpu() {row[0]:.3f} / {row[1]:.3f} / {row[2]:.3f} ms, .tolist() {tl:.3f} ms, "
          f"pinned non_blocking {tp:.3f} ms", flush=True)
