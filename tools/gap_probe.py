#!/usr/bin/env python3
"""Diagnostic: where does an MD step's wall time go outside the two kernels?  Times C2 MD steps
in windows shaped like the driver's bench call (--steps 20 --warmup 5) and longer ones, with and
without the HIP-event timing, and after an idle gap (clock ramp).

    python tools/gap_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import mdqtplasmasims_amd as M
    sim = M.Simulation(device=0, seed=12346, job=1, N0=3500).init()
    N = sim.N

    def window(steps, timing=0, idle=0.0):
        if idle:
            time.sleep(idle)
        sim.synchronize()
        if timing:
            sim.enable_timing(timing)
        t0 = time.perf_counter()
        sim.md_steps(steps)
        sim.synchronize()
        el = time.perf_counter() - t0
        f = s = None
        if timing:
            f_ms, nf, s_ms, ns = sim.kernel_time_totals()
            sim.enable_timing(False)
            f, s = f_ms / max(nf, 1) * 1e3, s_ms / max(ns, 1) * 1e3
        return el / steps * 1e6, f, s

    sim.md_steps(5)
    sim.synchronize()
    print(f"N={N}")
    for label, steps, timing, idle in [("20 steps, timing 8", 20, 8, 0), ("20 steps, no timing", 20, 0, 0),
                                       ("20 steps, after 0.5 s idle", 20, 0, 0.5),
                                       ("20 steps, timing 8, after 0.5 s idle", 20, 8, 0.5),
                                       ("200 steps, no timing", 200, 0, 0), ("200 steps, timing 8", 200, 8, 0),
                                       ("2000 steps, no timing", 2000, 0, 0),
                                       ("20 steps, no timing (hot)", 20, 0, 0),
                                       ("1 step x 20 (sync each)", 1, 0, 0)]:
        if label.startswith("1 step"):
            ts = [window(1)[0] for _ in range(20)]
            print(f"{label:40s} median {sorted(ts)[10]:8.2f} us per MD step (launch + sync round trip)")
            continue
        us, f, s = window(steps, timing, idle)
        extra = f" force {f:.2f} us, substeps {s:.2f} us, sum {f + s:.2f}" if f is not None else ""
        print(f"{label:40s} {us:8.2f} us per MD step{extra}")
    sim.close()


if __name__ == "__main__":
    main()
