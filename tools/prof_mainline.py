#!/usr/bin/env python3
"""Per-kernel durations of the bench's headline (C2) line inside a rocprofv3 --kernel-trace
database of the full `bench.py` command: the first K dispatches of each kernel (the headline line
runs first; later lines — pumping models, concurrent jobs_per_gpu streams, end-to-end — launch the
same kernel symbols, and the concurrent ones stretch their durations, so the whole-command
top_kernels average of a symbol is not the headline kernel's).

    python tools/prof_mainline.py gpurun_out/prof_r02/run_results.db 24 > profiles/<name>.txt
"""
import sqlite3
import sys


def main(db, k):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration from kernels order by start"))
    first = {}
    for name, dur in rows:
        first.setdefault(name, []).append(dur)
    print(f"# headline-line excerpt of {db.split('/')[-2]}: first {k} dispatches per kernel (durations in us)")
    print(f"{'n':>4} {'avg_us':>9} {'min_us':>9} {'max_us':>9}  kernel")
    for name, ds in first.items():
        if not any(t in name for t in ("k_substeps", "k_pairs_n3<", "k_pairs<")):
            continue
        ds = ds[:k]
        print(f"{len(ds):4d} {sum(ds) / len(ds) / 1e3:9.3f} {min(ds) / 1e3:9.3f} {max(ds) / 1e3:9.3f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
