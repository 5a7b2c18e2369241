#!/usr/bin/env python3
"""force_form_mode over a run (round 6): C5 (or another force_ab config) for K MD steps with QT, printing
every 10 steps the measured bound, the tiles recomputed so far, the model scale and the force time.

    python tools/form_drift.py C5 60 [opt=val,...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from force_ab import CFG  # noqa: E402


def main(cfg, k, opts=""):
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=12346, job=1, rng_mode=1, **CFG[cfg]).init()
    for o in filter(None, opts.split(",")):
        a, v = o.split("=")
        s.set_option(a, int(v))
    s.enable_timing(1, kinds=1)
    for i in range(0, k, 10):
        t0 = time.perf_counter()
        s.md_steps(10)
        s.synchronize()
        el = time.perf_counter() - t0
        f_ms, nf, _, _ = s.kernel_time_totals()
        print(f"{cfg} [{opts}] steps {i + 10}: {el / 10 * 1e3:.2f} ms/MD step, force {f_ms / max(nf, 1):.2f} ms; bound "
              f"{s.const('force_tail_bound'):.3e} raw {s.const('force_tail_raw_bound'):.3e} eps {s.const('force_error_eps'):.1e} "
              f"fixed {s.const('force_tail_fixed_tiles'):.0f} scale {s.const('force_tail_scale'):.0f} "
              f"r_far {s.const('force_far_radius'):.2f}", flush=True)
    s.close()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else "")
