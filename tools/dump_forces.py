#!/usr/bin/env python3
"""Forces of a library build (MDQT_LIB=...) at C2 and C5 (init() states) into an .npz, so that two builds
can be compared bit for bit (an A/B variant meant to change only the schedule, not the sums).

    MDQT_LIB=ab/x/libmdqt.so python tools/dump_forces.py out.npz
    python tools/dump_forces.py --compare a.npz b.npz
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path):
    import numpy as np
    import mdqtplasmasims_amd as M
    out = {}
    for name, kw in (("C2", dict(N0=3500)), ("C3", dict(N0=100000, Ge=1.0 / 12, qt_enabled=0)),
                     ("C5", dict(N0=250000, detuningDP=1.0))):
        s = M.Simulation(seed=12346, job=1, rng_mode=1, **kw).init()
        s.forces()
        out[name] = s.get_state()["F"]
        s.close()
    np.savez(path, **out)


def compare(a, b):
    import numpy as np
    A, B = np.load(a), np.load(b)
    for k in A.files:
        same = np.array_equal(A[k], B[k])
        d = np.abs(A[k] - B[k]).max() / np.abs(A[k]).max()
        print(f"{k}: bit-identical {same}, max|dF|/max|F| {d:.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
