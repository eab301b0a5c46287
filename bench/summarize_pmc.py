#!/usr/bin/env python3
"""Summarise bench/pmc_all.sh output: per kernel, counters averaged over dispatches,
plus derived ratios (MFMA busy share, wave-wait share, L2 hit rate, DRAM bytes)."""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 4, 8   # GRBM_GUI_ACTIVE is summed over the 8 XCDs


def load(root):
    per = defaultdict(lambda: defaultdict(list))
    files = glob.glob(os.path.join(root, "pmc_*_*", "run_counter_collection.csv"))
    files += glob.glob(os.path.join(root, "csv", "pmc_*_*.csv"))      # flattened copies
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "dalgo::" not in name and "kmeans_assign16" not in name:
                continue
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            per[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main(root):
    per = load(root)
    print("| kernel | MFMA busy % | wave wait % | VALU insts / wave | LDS bank confl / LDS inst | L2 hit % | DRAM rd GB (x2 calib.) |")
    print("|---|---|---|---|---|---|---|")
    for k, c in sorted(per.items()):
        a = {n: sum(v) / len(v) for n, v in c.items()}
        gui = a.get("GRBM_GUI_ACTIVE", 0)
        mfma = (100 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / XCDS * CUS * SIMDS)
                if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in a else float("nan"))
        wait = 100 * a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") else float("nan")
        valu = a["SQ_INSTS_VALU"] / a["SQ_WAVES"] if a.get("SQ_WAVES") and "SQ_INSTS_VALU" in a else float("nan")
        bank = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_INSTS_LDS"] if a.get("SQ_INSTS_LDS") else float("nan")
        hits, miss = a.get("TCC_HIT_sum"), a.get("TCC_MISS_sum")
        hit = 100 * hits / (hits + miss) if hits is not None and miss and hits + miss > 0 else float("nan")
        rd = a["TCC_EA0_RDREQ_sum"] * 64 * 2 / 1e9 if "TCC_EA0_RDREQ_sum" in a else float("nan")
        print(f"| `{k[:70]}` | {mfma:.1f} | {wait:.1f} | {valu:.0f} | {bank:.2f} | {hit:.1f} | {rd:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
