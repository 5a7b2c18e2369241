"""Where the end-to-end (reference cadence) time goes at C2: mdqt_run with and without outputs,
output() and writeConditions() alone, observables alone."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402


def run(sf, md=400):
    with tempfile.TemporaryDirectory() as d:
        s = M.Simulation(N0=3500, seed=12346, job=1, tmax=md * 0.002, sampleFreq=sf, saveDirectory=d + "/")
        s.init()
        t0 = time.perf_counter(); s.run(); s.synchronize(); el = time.perf_counter() - t0
        s.close()
    return el


def parts():
    with tempfile.TemporaryDirectory() as d:
        s = M.Simulation(N0=3500, seed=12346, job=1, saveDirectory=d + "/")
        s.init(); s.setup_directories(); s.md_steps(5); s.synchronize()
        r = {}
        for name, fn in [("observables", lambda: s.observables()), ("output", s.output),
                         ("writeConditions", lambda: s.writeConditions(5)), ("md_step", lambda: (s.md_steps(1), s.synchronize())),
                         ("get_state", s.get_state)]:
            fn()
            t0 = time.perf_counter()
            for _ in range(5):
                fn()
            r[name] = (time.perf_counter() - t0) / 5 * 1e3
        s.close()
    return r


run(40, 40)
print("run 400 MD steps, outputs every 40: %.1f ms" % (run(40) * 1e3))
print("run 400 MD steps, no outputs:       %.1f ms" % (run(100000) * 1e3))
print("per call (ms):", {k: round(v, 3) for k, v in parts().items()})
