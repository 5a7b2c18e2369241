#!/usr/bin/env python3
"""force_form_mode diagnostics (round 6): per configuration and option set, the tiers' radii, the census's
pair fractions by class, the measured error bound and the force-call time (HIP events, 3 calls).

    python tools/form_census.py "C5,C4,1M" "force_form_mode=1" "force_form_mode=0,force_mid_exp=11,..."
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from force_ab import CFG  # noqa: E402


def main(cfgs, optsets):
    import mdqtplasmasims_amd as M
    for cfg in cfgs.split(","):
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **CFG[cfg]).init()
        for opts in optsets:
            for o in filter(None, opts.split(",")):
                k, v = o.split("=")
                s.set_option(k, int(v))
            s.forces()
            s.synchronize()
            c = s.force_census()
            tot = sum(v[1] for v in c.values())
            s.enable_timing(1, kinds=1 | 2 | 8)
            for _ in range(3):
                s.forces()
            f_ms, nf, _, _ = s.kernel_time_totals()
            bd = s.force_breakdown()
            s.enable_timing(0)
            rad = {k: round(s.const(f"force_{k}_radius"), 2) for k in ("mid", "far", "vfar", "ufar", "ufar32")}
            print(f"{cfg} [{opts}] force {f_ms / nf:.3f} ms; r_t {s.const('force_skip_radius'):.2f} L/2 {s.const('L') / 2:.2f} "
                  f"radii {rad}; bound {s.const('force_tail_bound'):.3e} eps {s.const('force_error_eps'):.2e} "
                  f"fixed {s.const('force_tail_fixed_tiles'):.0f}", flush=True)
            print("    stages " + " ".join(f"{k} {bd[k]:.2f}" for k in ("sort_boxes", "plan", "block_kernel", "slot_reduce", "tail_pass")), flush=True)
            print("    " + " ".join(f"{k} {v[1] / tot:.4f}" for k, v in c.items() if v[1]), flush=True)
        s.close()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
