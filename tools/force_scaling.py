"""forces() time vs N (Newton-3 tiles below 65,536 ions, blocks above): is the C2 force kernel
throughput- or overhead-bound?  Prints N, us per call, pairs/s."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402

for N0 in [int(a) for a in (sys.argv[1:] or [1000, 2000, 3500, 5000, 8000, 16000, 32000, 60000, 100000])]:
    for scheme in ([2, 3] if N0 <= 60000 else [0]):
        s = M.Simulation(N0=N0, seed=12346).init()
        if scheme:
            s.set_option("force_scheme", scheme)
        for _ in range(5):
            s.forces()
        s.synchronize()
        s.enable_timing(1)
        n = 50 if N0 < 50000 else 10
        for _ in range(n):
            s.forces()
        s.synchronize()
        f_ms, nf, _, _ = s.kernel_time_totals()
        us = f_ms / nf * 1e3
        print(f"N={s.N:7d} scheme={scheme} {us:10.2f} us/call  {s.N * (s.N - 1) / 2 / us * 1e6:.3e} pairs/s", flush=True)
        s.close()
