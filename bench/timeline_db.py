#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 SQLite result: every dispatch in start order with its
duration and the idle gap before it (a long gap = the device waited on the host: a host
sync, a Python-side branch on a device value, or a first-launch code-object load).

usage: python bench/timeline_db.py <run_results.db> [--min-us X] [--skip N] [--limit N]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-us", type=float, default=0.0, help="hide kernels shorter than this")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--limit", type=int, default=100000)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if not rows:
        print("no kernels")
        return
    t0 = rows[0][1]
    prev_end = t0
    print("| # | t ms | gap us | dur us | kernel |")
    print("|---|---|---|---|---|")
    busy = 0
    for i, (n, s, e) in enumerate(rows):
        gap = (s - prev_end) / 1e3
        prev_end = max(prev_end, e)
        busy += e - s
        if i < a.skip or i >= a.skip + a.limit:
            continue
        if (e - s) / 1e3 < a.min_us and gap < 50:
            continue
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        print(f"| {i} | {(s - t0) / 1e6:.3f} | {gap:.1f} | {(e - s) / 1e3:.1f} | `{short}` |")
    span = (rows[-1][2] - t0) / 1e6
    print(f"\n{len(rows)} dispatches, span {span:.3f} ms, kernel busy {busy / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
