#!/usr/bin/env python3
"""C2 MD-step timing of one library build and engine options (A/B): init(), 20 warm MD steps, then
K MD steps between two synchronizations (wall clock), and the force / fused-substep launch averages
from HIP events.

    MDQT_AB_OPTS=force_tile_split=0 python tools/c2_step_ab.py NAME [K]
"""
import os
import sys
import time

ROOT = os.environ.get("MDQT_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(name, k=400):
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=12346, job=1, rng_mode=1, N0=3500).init()
    for o in filter(None, os.environ.get("MDQT_AB_OPTS", "").split(",")):
        opt, val = o.split("=")
        s.set_option(opt, int(val))
    s.md_steps(20)
    s.synchronize()
    t0 = time.perf_counter()
    s.md_steps(k)
    s.synchronize()
    dt = (time.perf_counter() - t0) / k
    s.enable_timing(1, kinds=3)
    s.md_steps(100)
    s.synchronize()
    t = s.kernel_times()
    s.enable_timing(0)
    s.close()
    print(f"{name}: C2 MD step {dt * 1e6:.2f} us, force {t['force_ms'] / max(t['n_force'], 1) * 1e3:.2f} us, "
          f"QT {t['substep_ms'] / max(t['n_substep'], 1) * 1e3:.2f} us", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 400)
