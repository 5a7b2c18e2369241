"""Diagnostic (variant build with -DMDQT_EXPT_MDSTAMPS): phases of the fused MD-step kernel at C2 —
force workgroups' start / end, QT workgroups' start / end of the wait / end.
    MDQT_LIB=expt/mdstamps/lib/libmdqt.so python tools/md_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402
from mdqtplasmasims_amd._lib import lib  # noqa: E402

s = M.Simulation(N0=3500, seed=12346).init()
s.set_option("fused_step", 1)
s.md_steps(6)
s.synchronize()
T = (s.N + 63) // 64
npairs = T * (T + 1) // 2
nq = (s.N + 15) // 16
n = npairs + nq
buf = (C.c_ulonglong * (4 * n))()
assert lib().mdqt_expt_md_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)
t0 = a[:, 0].min()
us = lambda x: (x - t0) * 10e-3
f, q = a[:npairs], a[npairs:]
pc = lambda v: np.percentile(v, [0, 10, 50, 90, 100]).round(2)
print(f"N={s.N} tile pairs {npairs}, QT workgroups {nq}")
print("force start", pc(us(f[:, 0])), " end", pc(us(f[:, 1])))
print("QT    start", pc(us(q[:, 0])), " wait done", pc(us(q[:, 2])), " end", pc(us(q[:, 1])))
s.close()
