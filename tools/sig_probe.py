"""Diagnostic: the Newton-3 tile kernel's time with the fused step's signalling (write-through slot
stores + per-tile arrival atomics) against plain, and the fused k_md_step launch, at C2.
    [MDQT_LIB=...] python tools/sig_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402

s = M.Simulation(N0=3500, seed=12346).init()
s.md_steps(5)
for label, fu, sig in (("plain", 0, 0), ("signalling", 0, 1), ("plain", 0, 0), ("fused", 1, 0)):
    s.set_option("fused_step", fu)
    s.set_option("expt_force_sig", sig)
    s.md_steps(3)
    s.synchronize()
    s.enable_timing(1, 3)
    s.md_steps(40)
    f_ms, nf, q_ms, nq = s.kernel_time_totals()
    s.enable_timing(0)
    print(f"{label:11s} force {f_ms / max(nf, 1) * 1e3:7.2f} us ({nf})  qt-kind {q_ms / max(nq, 1) * 1e3:7.2f} us ({nq})")
s.close()
