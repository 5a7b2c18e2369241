#!/usr/bin/env python3
"""Fused-substep launch timing of one library build (MDQT_LIB=...) at C5 and N = 1M, where the
thread-per-ion QT kernel runs (A/B of its variants): init(), one warm MD step, then K MD steps with
HIP events around every substep launch.

    MDQT_LIB=expt/<name>/lib/libmdqt.so python tools/qt_ab.py NAME [K]
"""
import os
import sys

ROOT = os.environ.get("MDQT_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = {"C5": dict(N0=250000, detuningDP=1.0), "1M": dict(N0=1000000)}


def main(name, k=3):
    import mdqtplasmasims_amd as M
    out = []
    for cfg, kw in CFG.items():
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **kw).init()
        s.md_steps(1)
        s.synchronize()
        s.enable_timing(1, kinds=2)
        s.md_steps(k)
        t = s.kernel_times()
        s.enable_timing(0)
        out.append(f"{cfg} {t['substep_ms'] / max(t['n_substep'], 1):.3f} ms")
        s.close()
    print(f"{name}: " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
