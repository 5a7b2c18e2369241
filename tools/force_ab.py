#!/usr/bin/env python3
"""Force-call timing of one library build (MDQT_LIB=...) at C3, C5 and N = 1M (A/B of block-kernel
variants; only API calls every round's library has): init(), one warm call, then K timed calls
(HIP events around each forces(): sort + block kernel + reduction).

    MDQT_LIB=expt/<name>/lib/libmdqt.so python tools/force_ab.py NAME [K]
    MDQT_AB_OPTS=force_ax1=0 python tools/force_ab.py NAME [K]      (engine options, comma-separated)
"""
import os
import sys

ROOT = os.environ.get("MDQT_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)      # MDQT_ROOT: another tree's package (an older round's library and wrapper)

CFG = {"C3": dict(N0=100000, Ge=1.0 / 12, qt_enabled=0), "C4": dict(N0=1000000, Ge=1.0 / 12, qt_enabled=0),
       "C5": dict(N0=250000, detuningDP=1.0),
       "1M": dict(N0=1000000), "C2": dict(N0=3500)}
DEFAULT = ("C3", "C5", "1M")


def main(name, k=3):
    import mdqtplasmasims_amd as M
    out = []
    only = os.environ.get("MDQT_AB_CFGS")      # e.g. "C5" (profiling one config), "C2,C3,C5,1M"
    for cfg, kw in CFG.items():
        if (only and cfg not in only.split(",")) or (not only and cfg not in DEFAULT):
            continue
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **kw).init()
        for o in filter(None, os.environ.get("MDQT_AB_OPTS", "").split(",")):   # e.g. "force_ax1=0"
            opt, val = o.split("=")
            s.set_option(opt, int(val))
        s.forces()
        s.synchronize()
        s.enable_timing(1, kinds=1)
        for _ in range(k if cfg != "C2" else 50 * k):
            s.forces()
        f_ms, nf, _, _ = s.kernel_time_totals()
        s.enable_timing(0)
        out.append(f"{cfg} {f_ms / max(nf, 1):.3f} ms" if cfg != "C2" else f"C2 {f_ms / max(nf, 1) * 1e3:.2f} us")
        s.close()
    print(f"{name}: " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
