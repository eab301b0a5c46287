"""K1 GPU-side cost vs sampled bytes: launches the production gradient kernel at several
row counts (10 % sampled, 1024 bf16 features) so a rocprofv3 kernel trace gives the
per-launch fixed cost (intercept) and the marginal streaming rate (slope), free of host
launch overhead. Run under: rocprofv3 --kernel-trace -d gpurun_out/k1i -o run
--output-format csv -- python3 bench/k1_intercept.py; then --parse DIR.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROWS = (20_000, 156_250, 312_500, 625_000, 1_250_000, 2_500_000, 5_000_000, 10_000_000)
REPS = 40


def run(a):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dalgo.ops import lr as L
    dev = torch.device("cuda", 0)
    Xall = torch.empty(max(ROWS), 1024, device=dev, dtype=torch.bfloat16).normal_()
    yall = (torch.rand(max(ROWS), device=dev) < 0.5).float()
    W = torch.zeros(1, 1025, device=dev)
    G = torch.zeros(1, 1025, device=dev)
    C = torch.zeros(1, device=dev)
    marker = torch.zeros(1, device=dev)
    for rows in ROWS:
        X, y = Xall[:rows], yall[:rows]
        seg = torch.tensor([0, rows], dtype=torch.int64, device=dev)
        for blocks in a.blocks:
          for fine in a.fine:
            marker.add_(1.0)          # separator kernel in the trace
            for i in range(REPS):
                L.lr_grad(X, y, W, seg, D=1024, frac=0.1, step=i, G=G, C=C,
                          target_blocks=blocks, g_is_zero=True, fine_groups=fine)
            torch.cuda.synchronize()
    print(json.dumps({"done": True, "rows": ROWS, "blocks": a.blocks}))


def parse(d, blocks, fines, pools=(0.0,)):
    rows_f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    recs = []
    for f in rows_f:
        for r in csv.DictReader(open(f)):
            recs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    recs.sort()
    # split at separator kernels (the torch add on `marker`)
    groups, cur = [], None
    for s, e, n in recs:
        if "lr_rows_kernel" in n:
            if cur is not None:
                cur.append((e - s) / 1e3)
        elif "OnSelf_add" in n:
            cur = []
            groups.append(cur)
    cfgs = [(r, b, f, 0.0) for r in ROWS for b in blocks for f in fines]
    out = []
    for (rows, b, f, pf), g in zip(cfgs, groups):
        g = sorted(g[5:]) if len(g) > 10 else sorted(g)
        med = g[len(g) // 2] if g else float("nan")
        gb = rows * 0.1 * 2048 / 1e9
        out.append({"rows": rows, "blocks": b, "fine": f, "pool": pf, "median_us": round(med, 2), "n": len(g),
                    "TBps": round(gb / (med * 1e-6) / 1e3, 2) if g else None})
        print(json.dumps(out[-1]))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--parse", default=None)
    ap.add_argument("--blocks", type=int, nargs="+", default=[256])
    ap.add_argument("--fine", type=int, nargs="+", default=[0])
    ap.add_argument("--rows", type=int, nargs="+", default=None)
    a = ap.parse_args()
    if a.rows:
        ROWS = tuple(a.rows)
    if a.parse:
        parse(a.parse, a.blocks, a.fine)
    else:
        run(a)
