"""Diagnostic (variant build with -DMDQT_EXPT_QTSTAMPS): where one fused substep launch of the lane
kernel spends its time per wave — prologue (loads, slot sum, Philox precompute, barrier), the
substep loop, the epilogue (stores).  MDQT_LIB=expt/qtstamps/lib/libmdqt.so python tools/qt_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402
from mdqtplasmasims_amd._lib import lib  # noqa: E402

s = M.Simulation(N0=int(sys.argv[1]) if len(sys.argv) > 1 else 3500, seed=12346).init()
s.md_steps(5)
s.synchronize()
s.forces()
s.substeps(25)
s.synchronize()
nw = (s.N + 3) // 4 // 4 * 4 + 4
nw = min(nw, 4096)
buf = (C.c_ulonglong * (16 * nw))()
lib().mdqt_expt_qt_stamps.argtypes = [C.c_void_p, C.c_int]
assert lib().mdqt_expt_qt_stamps(buf, nw) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
a = a[a[:, 0] > 0]
pro, loop, epi, tot = a[:, 1] - a[:, 0], a[:, 2] - a[:, 1], a[:, 3] - a[:, 2], a[:, 3] - a[:, 0]
rt = (a[:, 5] - a[:, 4]) * 10e-3          # us
clk = tot / rt / 1e3                        # GHz
t0 = a[:, 4].min()
print(f"N={s.N} waves={len(a)} span {((a[:, 5].max() - t0) * 10e-3):.2f} us; start spread "
      f"{((a[:, 4].max() - t0) * 10e-3):.2f} us; clock med {np.median(clk):.2f} GHz")
for name, v in (("prologue", pro), ("loop", loop), ("epilogue", epi), ("total", tot)):
    p = np.percentile(v, [0, 50, 100])
    print(f"{name:9s} cycles min/med/max {p[0]:9.0f} {p[1]:9.0f} {p[2]:9.0f}   med {p[1] / np.median(clk) / 1e3:6.2f} us")

for name, v in (("start -> loads issued", a[:, 9] - a[:, 0]), ("loads issued -> Philox done", a[:, 8] - a[:, 9]),
                ("Philox done -> force-slot sum", a[:, 6] - a[:, 8]), ("force-slot sum -> loop", a[:, 1] - a[:, 6]),
                ("prologue to the force-slot sum (loads + Philox)", a[:, 6] - a[:, 0])):
    p = np.percentile(v, [0, 50, 100])
    print(f"{name:48s} min/med/max {p[0]:6.0f} {p[1]:6.0f} {p[2]:6.0f}")
nj = a[:, 7]
for j in range(int(nj.max()) + 1):
    m = nj == j
    if m.any():
        print(f"waves with {j} jump substeps: {m.sum():4d}  loop cycles med {np.median(loop[m]):8.0f} max {loop[m].max():8.0f}")
