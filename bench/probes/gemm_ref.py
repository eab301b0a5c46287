"""Library GEMM reference points on this MI355X: torch._int_mm (int8 -> int32) and bf16
matmul at n = 16384 (the K9 closure step's shape), for calibrating the hand-written K9."""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


n = 16384
dev = torch.device("cuda", 0)
a8 = torch.randint(0, 2, (n, n), dtype=torch.int8, device=dev)
b8 = torch.randint(0, 2, (n, n), dtype=torch.int8, device=dev)
out = {}
try:
    dt = timed(lambda: torch._int_mm(a8, b8.t()))
    out["int_mm_ms"] = dt * 1e3
    out["int_mm_TOPs"] = 2 * n ** 3 / dt / 1e12
except Exception as e:  # noqa: BLE001
    out["int_mm_error"] = repr(e)[:200]
ab = torch.randn(n, n, dtype=torch.bfloat16, device=dev)
bb = torch.randn(n, n, dtype=torch.bfloat16, device=dev)
dt = timed(lambda: ab @ bb.t())
out["bf16_mm_ms"] = dt * 1e3
out["bf16_mm_TFLOPs"] = 2 * n ** 3 / dt / 1e12
print(json.dumps(out), flush=True)
