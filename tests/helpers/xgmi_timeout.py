"""torchrun helper: force a K11 peer-flag timeout on rank 0 only (rank 1 never joins
the exchange) and check that the collective error check raises on EVERY rank and
that runtime.shutdown() then exits non-zero."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.parallel import comm, runtime, xgmi  # noqa: E402


def main():
    os.environ["DALGO_XGMI"] = "1"
    rt = runtime.init(backend="gloo", device="cuda", app_name="xgmi-timeout")
    xg = xgmi.shared(rt.device)
    assert xg is not None, "xGMI all-reduce did not come up"
    xg.timeout_s = 0.5
    if rt.rank == 0:
        x = torch.ones(64, device=rt.device)
        xg.all_reduce_(x)          # rank 1 never pushes: the bounded wait expires
    torch.cuda.synchronize()
    try:
        comm.check_device_errors("forced timeout")
        print(f"XG_NO_RAISE rank {rt.rank}", flush=True)
    except comm.DeviceCollectiveError:
        print(f"XG_RAISED rank {rt.rank}", flush=True)
    runtime.shutdown()             # must raise SystemExit(3)
    print(f"XG_SHUTDOWN_RETURNED rank {rt.rank}", flush=True)


if __name__ == "__main__":
    main()
