"""Quick timing of the MCMD engine stages on the GPU (N = 4096), beside the reference on 1 core."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdqtplasmasims_amd import mdmc  # noqa: E402


def main():
    tmp = tempfile.mkdtemp()
    e = mdmc.MonteCarloMD(seed=3, saveDirectory=tmp + "/")
    e.init()
    e.monte_carlo(1000)
    t = time.perf_counter(); n = 20000; acc = e.monte_carlo(n); dt = time.perf_counter() - t
    print(f"MC: {n / dt:.0f} steps/s ({dt / n * 1e6:.2f} us/step), acceptance {acc / n:.3f}", flush=True)
    e.md_steps(50)
    for cf in (0.0, 0.25):
        e.set_collision_freq(cf)
        t = time.perf_counter(); n = 2000; e.md_steps(n); dt = time.perf_counter() - t
        print(f"MD (collisionFreq {cf}): {n / dt:.0f} steps/s ({dt / n * 1e6:.2f} us/step)", flush=True)
    t = time.perf_counter(); g = e.pair_corr(); dt = time.perf_counter() - t
    print(f"g(r): {dt * 1e3:.2f} ms", flush=True)
    import numpy as np
    vs = np.random.default_rng(1).normal(0, 0.5, (3, 4096, 2500))
    e.set_velocity_store(vs)
    e.autocorrelations()
    t = time.perf_counter(); e.autocorrelations(); dt = time.perf_counter() - t
    print(f"autocorrelations T=2500: {dt * 1e3:.2f} ms", flush=True)
    if "--ref" in sys.argv:
        from oracle import oracle as O
        r = O.RefMCMD(seed=3, save_directory=tmp + "/")
        r.init()
        t = time.perf_counter(); n = 2000; r.monte_carlo(n); dt = time.perf_counter() - t
        print(f"reference MC (1 core): {n / dt:.0f} steps/s", flush=True)
        t = time.perf_counter(); n = 3; r.md_steps(n); dt = time.perf_counter() - t
        print(f"reference MD (1 core): {n / dt:.2f} steps/s", flush=True)


if __name__ == "__main__":
    main()
