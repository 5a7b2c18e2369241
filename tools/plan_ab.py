#!/usr/bin/env python3
"""Force-call stage timing of one library build (MDQT_LIB=...) at the large configurations, with a
digest of the forces so that builds meant to be bit-identical can be checked against each other
(A/B of the plan kernel k_n3b_plan, round 6):

    MDQT_LIB=expt/<name>/lib/libmdqt.so python tools/plan_ab.py NAME [K]
    MDQT_AB_CFGS=C5,1M python tools/plan_ab.py NAME

Prints per configuration the plan stage, the block kernel and the whole force call (ms, events between
the stages, force_breakdown) and the first 16 hex digits of sha256 over F after the timed calls."""
import hashlib
import os
import sys

ROOT = os.environ.get("MDQT_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = {"C3": dict(N0=100000, Ge=1.0 / 12, qt_enabled=0), "C4": dict(N0=1000000, Ge=1.0 / 12, qt_enabled=0),
       "C5": dict(N0=250000, detuningDP=1.0), "1M": dict(N0=1000000)}


def main(name, k=3):
    import mdqtplasmasims_amd as M
    cfgs = os.environ.get("MDQT_AB_CFGS", "C3,C5,1M").split(",")
    for cfg in cfgs:
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **CFG[cfg]).init()
        s.forces()
        s.synchronize()
        s.enable_timing(1, kinds=1 | 8)
        for _ in range(k):
            s.forces()
        s.synchronize()
        bd = s.force_breakdown()
        s.enable_timing(0)
        dig = hashlib.sha256(s.get_state()["F"].tobytes()).hexdigest()[:16]
        print(f"{name} {cfg} plan {bd['plan']:.3f} kernel {bd['block_kernel']:.3f} force {bd['forces_total']:.3f} ms"
              f" F {dig}", flush=True)
        s.close()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
