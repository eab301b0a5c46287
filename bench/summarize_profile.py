#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv (+ per-kernel VGPR/LDS from the trace) as markdown."""
import csv
import sys
from collections import defaultdict


def main(d, top=14):
    stats = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    res = {}
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        res.setdefault(r["Kernel_Name"], (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"],
                                          r["Grid_Size_X"], r["Workgroup_Size_X"]))
    print("| kernel | calls | avg us | total % | VGPR | LDS B | grid x wg |")
    print("|---|---|---|---|---|---|---|")
    for r in stats[:top]:
        n = r["Name"]
        v = res.get(n, ("?", "?", "?", "?", "?"))
        short = n.replace("void ", "")[:80]
        print(f"| `{short}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} | {v[0]} | {v[2]} | {v[3]}x{v[4]} |")


if __name__ == "__main__":
    main(sys.argv[1])
