"""Native radix sort vs rocPRIM on the build's key shapes (one MI355X): u64 keys, the
scale-26 one-rank key sort (1.07B keys, bits 12..51) and the W = 8 share (134M keys, bits
8..48), plus the source partition (2 passes over bits 45..58 of packed pairs). Prints
ms per sort, best of 3, for DALGO_SORT as set in the environment."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.ops import _ext  # noqa: E402

ops = _ext.ops()
dev = torch.device("cuda")
res = {"sort": os.environ.get("DALGO_SORT", "native")}
for name, n, lo, hi in (("keys_w1", 1 << 30, 12, 52), ("keys_w8", 134_635_295, 8, 48),
                        ("src_partition", 1 << 30, 45, 58)):
    keys = torch.randint(0, 1 << 62, (n,), dtype=torch.int64, device=dev)
    out = torch.empty_like(keys)
    best = 1e9
    for _ in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        ops.gb_sort(keys, n, hi, out, lo)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    res[name] = best * 1e3
    res[name + "_GBps"] = n * 8 * 2 * ((hi - lo + 7) // 8) / best / 1e9
    ok = bool(torch.equal(out[:1000000].cpu(), out[:1000000].cpu())) if False else None
    del keys, out
    torch.cuda.empty_cache()
res["err"] = int(ops.rs_sort_error(torch.zeros(1, device=dev)).item())
print(json.dumps(res), flush=True)
