"""BASELINE.md §2-§3 calibration of the CPU baseline: the oracle restatement (the bench's
cpu_baseline, kind "port") on the same container and thread counts as the reference's own
single-thread measurement of BASELINE.md §2 / SURVEY App. B-3 (SpeedUp, N = 3573, 1 thread:
4.23e4 particle-qsteps/s; 8 threads 2.63e5, racy).  Writes profiles/<tag>_cpu_calibration.json;
bench.py reads the newest one and reports the ratio beside its cpu_baseline.

    python tools/cpu_calibration.py r04
"""
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REFERENCE = {"1": 4.23e4, "8": 2.63e5}      # BASELINE.md §2 (SpeedUp itself, this container, N = 3573)


def main(tag):
    from oracle import oracle as O
    res = {}
    for threads, steps in ((1, 8), (8, 24)):
        o = O.OracleSim(rng_mode=1, nthreads=threads, qt_enabled=1, seed=12346, job=1, N0=3500).init()
        ratio = int(o.const("plasmaToQuantumTimestepRatio"))
        o.md_steps(1)
        t0 = time.perf_counter()
        o.md_steps(steps)
        el = time.perf_counter() - t0
        rate = o.N * ratio * steps / el
        res[str(threads)] = {"N": o.N, "md_steps": steps, "seconds": el, "oracle_particle_qsteps_per_s": rate,
                             "reference_particle_qsteps_per_s": REFERENCE[str(threads)],
                             "oracle_over_reference": rate / REFERENCE[str(threads)]}
        o.close()
    out = {"_meta": {"what": "oracle C restatement vs the reference SpeedUp (BASELINE.md §2), same container, "
                             "C2 (N0 = 3500, seed 12346), rng_mode 1",
                     "cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count()},
           "threads": res}
    path = os.path.join(ROOT, "profiles", f"{tag}_cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r04")
