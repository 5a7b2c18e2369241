"""Diagnostic (variant build with -DMDQT_EXPT_STAMPS): per-workgroup start/end times and placement
of the Newton-3 tile kernel at C2.  MDQT_LIB=expt/stamps/lib/libmdqt.so python tools/n3_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdqtplasmasims_amd as M  # noqa: E402
from mdqtplasmasims_amd._lib import lib  # noqa: E402

s = M.Simulation(N0=int(sys.argv[1]) if len(sys.argv) > 1 else 3500, seed=12346).init()
for _ in range(3):
    s.md_steps(1)
s.synchronize()
s.forces()
s.synchronize()
ntiles = (s.N + 63) // 64
k = int(s.const("force_tile_split_pairs"))         # the split table's extra workgroups (halves)
n = ntiles * (ntiles + 1) // 2 + (k if s.const("force_tile_split") == 1 else 0)
buf = (C.c_ulonglong * (6 * n))()
assert lib().mdqt_expt_n3_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 6).astype(np.int64)
t0 = a[:, 0].min()
st = (a[:, 0] - t0) * 10e-3      # us (100 MHz)
en = (a[:, 1] - t0) * 10e-3
life = en - st
hw = a[:, 2]
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
xcc = a[:, 3] & 15
print(f"N={s.N} WGs={n} kernel span {en.max():.2f} us")
print("start  pct 0/10/50/90/100:", np.percentile(st, [0, 10, 50, 90, 100]).round(2))
print("end    pct 0/10/50/90/100:", np.percentile(en, [0, 10, 50, 90, 100]).round(2))
print("life   pct 0/10/50/90/100:", np.percentile(life, [0, 10, 50, 90, 100]).round(2))
key = xcc * 1000 + se * 100 + sh * 16 + cu
u, cnt = np.unique(key, return_counts=True)
print("distinct CUs used:", len(u), " WGs per CU min/mean/max:", cnt.min(), round(cnt.mean(), 2), cnt.max())
print("per-XCC WGs:", np.bincount(xcc, minlength=8))
diag = np.array([0])
hist = np.histogram(st, bins=10)[0]
clk = (a[:, 5] - a[:, 4]) / np.maximum(a[:, 1] - a[:, 0], 1) * 100e6 / 1e9
print("core clock GHz (s_memtime / s_memrealtime) pct 0/50/100:", np.percentile(clk, [0, 50, 100]).round(3))
print("start histogram (10 bins over span):", hist)
# per-CU end times grouped by the number of workgroups the CU ran
last = {}
for kk, e, c in zip(key, en, np.ones_like(en)):
    last.setdefault(kk, []).append(e)
by = {}
for kk, es in last.items():
    by.setdefault(len(es), []).append(max(es))
for nwg, ends in sorted(by.items()):
    print(f"CUs with {nwg} WGs: {len(ends)}, last end pct 0/50/100:", np.percentile(ends, [0, 50, 100]).round(2))
# dispatch order: start time against the workgroup index (the tile-pair list order)
idx = np.arange(n)
for q in range(0, n, max(n // 8, 1)):
    sl = slice(q, min(q + n // 8, n))
    print(f"blocks {q:5d}..{min(q + n // 8, n) - 1:5d}: start med {np.median(st[sl]):.2f} max {st[sl].max():.2f}  "
          f"end med {np.median(en[sl]):.2f} max {en[sl].max():.2f}")
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/n3_stamps_raw.npy", a)
