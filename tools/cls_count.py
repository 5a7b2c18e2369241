"""Diagnostic (variant build with -DMDQT_EXPT_CLS): fractions of the Newton-3 block kernel's tile
pairs that are skipped, take the uniform minimum image, or the per-pair one, at C3 / C5 / N=1M.
MDQT_LIB=expt/cls/lib/libmdqt.so python tools/cls_count.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402
from mdqtplasmasims_amd._lib import lib  # noqa: E402

buf = (C.c_ulonglong * 3)()
for name, kw in [("C3", dict(N0=100000, Ge=1.0 / 12, qt_enabled=0)), ("C5", dict(N0=250000, detuningDP=1.0)),
                 ("1M", dict(N0=1000000))]:
    s = M.Simulation(seed=12346, **kw).init()
    lib().mdqt_expt_cls_count(buf, 1)
    s.forces()
    s.synchronize()
    lib().mdqt_expt_cls_count(buf, 1)
    tot = sum(buf)
    print(f"{name}: N={s.N} tile-pair classes (x BW waves each counted once per J): skip {buf[0] / tot:.3f} "
          f"per-pair {buf[1] / tot:.3f} uniform {buf[2] / tot:.3f}")
    s.close()
