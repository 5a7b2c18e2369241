#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (one rocpd database per pass).

    python tools/pmc_summary.py gpurun_out/pmc_fetch/run_results.db gpurun_out/pmc_write/run_results.db ...
        [--factors FETCH WRITE] [--trace gpurun_out/trace/run_results.db] [--tag NAME]

Counter values are summed over the rows of one dispatch (per-SE / per-XCD instances), then
averaged over the dispatches of each kernel.  Prints JSON {kernel: {counter: mean, "dispatches": n}}.
With --trace (a --kernel-trace database of the same command, un-profiled counters) each kernel also
gets its average dispatch duration "duration_us"; --tag records what workload the passes ran.
"""
import collections
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(db):
    c = sqlite3.connect(db)
    per = collections.defaultdict(float)   # (kernel, dispatch, counter) -> value
    for k, d, n, v in c.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
        per[(k, d, n)] += v
    return per


def main(args):
    """args: the rocpd databases, then optionally --factors FETCH_FACTOR WRITE_FACTOR (the
    calibration of tools/fetch_calib.hip for the kernel's access pattern)"""
    from bench import kernel_source_hash
    meta = {"src_hash": kernel_source_hash()}
    dbs = list(args)
    if "--factors" in dbs:
        k = dbs.index("--factors")
        meta["fetch_factor"], meta["write_factor"] = float(dbs[k + 1]), float(dbs[k + 2])
        dbs = dbs[:k] + dbs[k + 3:]
    trace = None
    if "--trace" in dbs:
        k = dbs.index("--trace")
        trace = dbs[k + 1]
        dbs = dbs[:k] + dbs[k + 2:]
    if "--tag" in dbs:
        k = dbs.index("--tag")
        meta["workload"] = dbs[k + 1]
        dbs = dbs[:k] + dbs[k + 2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for db in dbs:
        for (k, d, n), v in load(db).items():
            agg[k][n].append(v)
    out = {"_meta": meta}
    for k, cs in agg.items():
        out[k] = {n: sum(v) / len(v) for n, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    if trace:
        c = sqlite3.connect(trace)
        for name, calls, avg in c.execute("select name, total_calls, average from top_kernels"):
            if name in out:
                out[name]["duration_us"] = avg                  # top_kernels: microseconds (tools/prof_summary.py)
                out[name]["trace_dispatches"] = calls
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
