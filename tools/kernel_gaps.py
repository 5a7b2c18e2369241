#!/usr/bin/env python3
"""Inter-kernel gaps from a rocprofv3 --kernel-trace database (rocpd sqlite).

    python tools/kernel_gaps.py gpurun_out/prof_drv/run_results.db [--last K]

Prints the dispatch sequence of the last K kernels (default 60) with each kernel's duration
and the idle gap before it, then the median gap per (previous kernel -> kernel) transition."""
import sqlite3
import statistics
import sys
from collections import defaultdict


def rows(db):
    c = sqlite3.connect(db)
    for q in ("select name, start, end from kernels order by start",
              "select kernel_name, start, end from kernels order by start"):
        try:
            return list(c.execute(q))
        except sqlite3.Error:
            continue
    print("no kernels view; schema:")
    for (n, s) in c.execute("select name, sql from sqlite_master"):
        print(n, (s or "")[:200])
    sys.exit(1)


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("mdqt::", "")
    return n[:48]


def main():
    db = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 60
    r = rows(db)
    print(f"{len(r)} kernels")
    tail = r[-last:]
    trans = defaultdict(list)
    prev = None
    for name, s, e in r:
        if prev is not None:
            trans[(short(prev[0]), short(name))].append((s - prev[2]) / 1e3)
        prev = (name, s, e)
    print(f"{'gap_us':>9} {'dur_us':>9}  kernel")
    p = None
    for name, s, e in tail:
        g = (s - p) / 1e3 if p is not None else 0.0
        print(f"{g:9.2f} {(e - s) / 1e3:9.2f}  {short(name)}")
        p = e
    print("\nmedian gap per transition (us), count")
    for k, v in sorted(trans.items(), key=lambda kv: -len(kv[1])):
        print(f"{statistics.median(v):9.2f} {len(v):6d}  {k[0]} -> {k[1]}")
    durs = defaultdict(list)
    for name, s, e in r:
        durs[short(name)].append((e - s) / 1e3)
    print("\nmedian duration per kernel (us), count")
    for k, v in sorted(durs.items(), key=lambda kv: -len(kv[1])):
        print(f"{statistics.median(v):9.2f} {len(v):6d}  {k}")


if __name__ == "__main__":
    main()
