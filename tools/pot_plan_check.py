#!/usr/bin/env python3
"""Epotential() on the Newton-3 blocks: the force call's plan (option potential_plan 1, round 6) against
every pair to L/2 in the exact form (0) — values and the block kernel's time in each mode, beside the
force call's (timing kinds: bit 0 forces, bit 2 the potential calls' block kernel).

    python tools/pot_plan_check.py [C3,C5,C4,1M] [K]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CFG = {"C3": dict(N0=100000, Ge=1.0 / 12, qt_enabled=0), "C4": dict(N0=1000000, Ge=1.0 / 12, qt_enabled=0),
       "C5": dict(N0=250000, detuningDP=1.0), "1M": dict(N0=1000000)}


def main(cfgs, k=2):
    import mdqtplasmasims_amd as M
    res = {}
    for cfg in cfgs:
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **CFG[cfg]).init()
        s.md_steps(1)
        r = {"N": s.N}
        s.enable_timing(1, kinds=1 | 4)
        for _ in range(k):
            s.forces()
        for mode in (1, 0):
            s.set_option("potential_plan", mode)
            s.synchronize()
            t0 = time.perf_counter()
            e = [s.Epotential() for _ in range(k)]
            s.synchronize()
            wall = (time.perf_counter() - t0) / k
            kt = s.kernel_times()
            r[f"plan{mode}"] = {"Epot": e[-1], "wall_ms": wall * 1e3,
                                "pot_block_ms": kt["pot_block_ms"] / max(kt["n_pot_block"], 1)}
            if mode == 1:
                r["force_ms"] = kt["force_ms"] / max(kt["n_force"], 1)
                r["force_block_ms"] = kt["block_ms"] / max(kt["n_block"], 1)
        r["rel_diff"] = abs(r["plan1"]["Epot"] - r["plan0"]["Epot"]) / abs(r["plan0"]["Epot"])
        s.close()
        res[cfg] = r
        print(cfg, json.dumps(r), flush=True)
    return res


if __name__ == "__main__":
    main(sys.argv[1].split(",") if len(sys.argv) > 1 else ["C3", "C5", "1M"], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
