#!/usr/bin/env python3
"""mdqt_run() end to end at C5 (bench.py's end_to_end_c5 recipe: run to 80 MD steps minus run to 40, files
written) with options per run, and the time of each output() stage (round 6 diagnostics)

    python tools/e2e_form.py "force_form_mode=1" "force_form_mode=0"
"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(steps, opts):
    import mdqtplasmasims_amd as M
    with tempfile.TemporaryDirectory() as d:
        sim = M.Simulation(seed=12346, job=1, N0=250000, detuningDP=1.0, tmax=steps * 0.002, saveDirectory=d + "/")
        for o in filter(None, opts.split(",")):
            a, v = o.split("=")
            sim.set_option(a, int(v))
        t0 = time.perf_counter()
        sim.run()
        sim.synchronize()
        el = time.perf_counter() - t0
        c0 = sim.counters()["c0"]
        sim.close()
    return el, c0


def main(optsets):
    one(40, optsets[0])
    for opts in optsets:
        (a, ca), (b, cb) = one(40, opts), one(80, opts)
        print(f"[{opts}] {(b - a) / (cb - ca) * 1e3:.2f} ms per MD step (runs {a:.3f} s / {b:.3f} s)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
