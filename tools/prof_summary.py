#!/usr/bin/env python3
"""Dump the per-kernel summary (top_kernels view) of a rocprofv3 rocpd database as text.

    python tools/prof_summary.py gpurun_out/prof1/run_results.db > profiles/<name>.txt
"""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    cur = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    print(f"# rocprofv3 --kernel-trace --stats summary of {db.split('/')[-2]} (durations in us)")
    print(f"{'calls':>7} {'total_us':>12} {'avg_us':>10} {'pct':>6}  kernel")
    for name, calls, tot, avg, pct in cur:
        print(f"{calls:7d} {tot:12.3f} {avg:10.3f} {pct:6.2f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
