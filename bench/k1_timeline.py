"""K1 per-wave timeline (diagnostics): where the fixed ~12-15 us of a gradient launch goes.

Every wave of one production-shape K1 launch records s_memrealtime (100 MHz) at start, at
its first row batch issued, at the end of its sweep and (block leader) after its epilogue
atomics, plus its selected-row count and CU id (csrc/kernels/lr_grad.hip, `trace`).
Printed per row count: dispatch ramp, start-up latency, sweep-finish spread, epilogue
time, and the block-level row imbalance against the finish order.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalgo.ops import _ext  # noqa: E402
from dalgo.ops import lr as L  # noqa: E402

NW = 8   # waves per block of the default variant (3)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def main():
    dev = torch.device("cuda", 0)
    ops = _ext.ops()
    args = sys.argv[1:]
    fines = [0]
    frac = 0.1
    if "--frac" in args:
        i = args.index("--frac")
        frac = float(args[i + 1])
        args = args[:i] + args[i + 2:]
    use_list = "--list" in args
    if use_list:
        args = [x for x in args if x != "--list"]
    if "--fine" in args:
        i = args.index("--fine")
        fines = [int(x) for x in args[i + 1:]]
        args = args[:i]
    rows_list = [int(x) for x in (args or ["20000", "1250000", "10000000"])]
    Xall = torch.empty(max(rows_list), 1024, device=dev, dtype=torch.bfloat16).normal_()
    yall = (torch.rand(max(rows_list), device=dev) < 0.5).float()
    W = torch.zeros(1, 1025, device=dev)
    G = torch.zeros(1, 1025, device=dev)
    C = torch.zeros(1, device=dev)
    buf = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    for rows, fine in [(r, f) for r in rows_list for f in fines]:
        X, y = Xall[:rows], yall[:rows]
        seg = torch.tensor([0, rows], dtype=torch.int64, device=dev)
        gx, _ = L._grid(rows, 1)
        res = []
        for rep in range(6):
            for i in range(5):
                L.lr_grad(X, y, W, seg, D=1024, frac=frac, step=100 * rep + i, G=G, C=C, g_is_zero=True,
                          fine_groups=fine)
            buf.zero_()
            torch.cuda.synchronize()
            ops.lr_set_trace(buf)
            L.lr_grad(X, y, W, seg, D=1024, frac=frac, step=100 * rep + 50, G=G, C=C, g_is_zero=True,
                      fine_groups=fine)
            ops.lr_set_trace(None)
            torch.cuda.synchronize()
            t = buf[: gx * NW * 8].view(gx, NW, 8).cpu().double()
            t0 = t[:, :, 0].min().item()
            us = lambda v: (v - t0) / 100.0   # noqa: E731
            start = us(t[:, :, 0]).flatten().tolist()
            first = (t[:, :, 1] - t[:, :, 0]).flatten().div(100.0).tolist()
            bar = (t[:, :, 6] - t[:, :, 0]).flatten().div(100.0).tolist()
            refl = (t[:, :, 7] - t[:, :, 0]).flatten().div(100.0).tolist()
            done = us(t[:, :, 2]).flatten().tolist()
            epi_end = us(t[:, 0, 3]).tolist()
            epi = ((t[:, 0, 3] - t[:, :, 2].max(dim=1).values) / 100.0).tolist()
            brows = t[:, :, 4].sum(dim=1)
            bdone = us(t[:, :, 2].max(dim=1).values)
            order = torch.argsort(bdone)
            intra = ((t[:, :, 2].max(dim=1).values - t[:, :, 2].min(dim=1).values) / 100.0).tolist()
            bd = bdone.tolist()
            last8 = brows[order[-8:]].mean().item()
            # blocks are dealt round-robin over the 8 XCDs: per-XCD medians of the block
            # finish time and of the time per selected row
            per_row = (bdone - us(t[:, :, 0].min(dim=1).values)) / brows.clamp(min=1)
            xcd_done = [bdone[i::8].median().item() for i in range(8)]
            xcd_rate = [per_row[i::8].median().item() * 1e3 for i in range(8)]
            bc = torch.stack([bdone - bdone.mean(), brows - brows.mean()])
            corr = (bc[0] * bc[1]).sum() / (bc[0].norm() * bc[1].norm() + 1e-12)
            res.append({
                "start_p50": pct(start, 0.5), "start_max": max(start),
                "barrier_p50": pct(bar, 0.5), "refill_p50": pct(refl, 0.5),
                "first_issue_p50": pct(first, 0.5), "first_issue_max": max(first),
                "sweep_done_p10": pct(done, 0.1), "sweep_done_p50": pct(done, 0.5),
                "sweep_done_p90": pct(done, 0.9), "sweep_done_max": max(done),
                "intra_block_spread_p50": pct(intra, 0.5), "intra_block_spread_p90": pct(intra, 0.9),
                "block_done_p10": pct(bd, 0.1), "block_done_p50": pct(bd, 0.5), "block_done_max": max(bd),
                "epilogue_p50": pct(epi, 0.5), "epilogue_max": max(epi), "end_max": max(epi_end),
                "block_rows_mean": brows.mean().item(), "block_rows_max": brows.max().item(),
                "rows_last8_blocks": last8,
                "wave_rows_max": t[:, :, 4].max().item(),
                "xcd_done_spread": max(xcd_done) - min(xcd_done),
                "xcd_ns_per_row_min": min(xcd_rate), "xcd_ns_per_row_max": max(xcd_rate),
                "ns_per_row_cv": (per_row.std() / per_row.mean()).item(),
                "corr_done_rows": corr.item(),
                "cus": len(set(t[:, :, 5].flatten().tolist())),
            })
        med = {k: round(sorted(r[k] for r in res)[len(res) // 2], 2) for k in res[0]}
        print(json.dumps({"rows": rows, "frac": frac, "fine": fine, "list": use_list, "blocks": gx, **med}), flush=True)


if __name__ == "__main__":
    main()
