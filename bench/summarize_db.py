#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite result (default output format) as a markdown kernel table.

usage: python bench/summarize_db.py <run_results.db> [top]
"""
import sqlite3
import sys


def main(path, top=12):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), avg(end-start), sum(end-start), max(vgpr_count), max(lds_size),"
        " max(grid_x), max(workgroup_x) from kernels group by name order by sum(end-start) desc").fetchall()
    tot = sum(r[3] for r in rows) or 1
    print("| kernel | calls | avg us | total % | VGPR | LDS B | grid x wg |")
    print("|---|---|---|---|---|---|---|")
    for n, k, avg, s, vg, lds, gx, wx in rows[:top]:
        short = n.replace("void ", "")[:80]
        print(f"| `{short}` | {k} | {avg / 1e3:.1f} | {100 * s / tot:.1f} | {vg} | {lds} | {gx}x{wx} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
