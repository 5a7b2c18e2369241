#!/usr/bin/env python3
"""The block kernel's lock-step J loop: estimated VALU per J step over a workgroup's 8 waves, busiest wave
against the mean (mdqt_force_jstep_balance), for the large configs' init() states.

    python tools/jstep_balance.py [C3,C5,C4,1M]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CFG = {"C3": dict(N0=100000, Ge=1.0 / 12, qt_enabled=0), "C4": dict(N0=1000000, Ge=1.0 / 12, qt_enabled=0),
       "C5": dict(N0=250000, detuningDP=1.0), "1M": dict(N0=1000000)}


def main(cfgs):
    import mdqtplasmasims_amd as M
    for cfg in cfgs:
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **CFG[cfg]).init()
        b = s.force_jstep_balance()
        print(cfg, json.dumps(b), flush=True)
        s.close()


if __name__ == "__main__":
    main(sys.argv[1].split(",") if len(sys.argv) > 1 else ["C3", "C5", "C4", "1M"])
