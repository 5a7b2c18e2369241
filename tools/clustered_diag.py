#!/usr/bin/env python3
"""Diagnostic (GPU): the clustered N = 1M case of tests/test_gpu_large.py — which ions differ most
between the tail-only forces (C) and the exact-order sum (E), and how both compare with the exact
sum in long double over all partners inside L/2 (X).  Separates the tail (|C - X|) from the
summation rounding (|E - X|); it found k_tail_fix's plain 1e5-term chain.

    python tools/clustered_diag.py
"""
import os
import sys

import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_large import clustered_state, CLUSTERED, SEED
import mdqtplasmasims_amd as M
N0, k, frac, rc = CLUSTERED["1M"]
eps = 10.0 ** -k
s = M.Simulation(N0=N0, seed=SEED, job=1, rng_mode=1)
L = s.const("L"); lD = s.const("lDeb")
state = clustered_state(N0, L, frac, rc)
s.set_state(*state)
s.set_option("force_tail_exp", k)
for o in ("force_mid_exp", "force_far_exp", "force_vfar_exp", "force_ufar_exp"):
    s.set_option(o, 0)
s.forces(); C = s.get_state()["F"]
print("fixed tiles", s.const("force_tail_fixed_tiles"), "rt", s.const("force_skip_radius"), flush=True)
s.set_option("force_tail_exp", 0)
s.forces(); E = s.get_state()["F"]
s.close()
R = state[0]
d = np.abs(C - E).max(axis=0)
idx = np.argsort(d)[::-1][:12]
ctr = L / 2
for i in idx:
    dr = R[:, i:i + 1] - R
    dr -= L * np.round(dr / L)
    r = np.sqrt((dr.astype(np.longdouble) ** 2).sum(axis=0))
    m = (r > 0) & (r < L / 2)
    rr = r[m]
    ft = (1 / rr + 1 / np.longdouble(lD)) * np.exp(-rr / np.longdouble(lD)) / rr ** 2
    X = (dr[:, m].astype(np.longdouble) * ft).sum(axis=1)
    rb = np.sqrt(((R[:, i] - ctr) ** 2).sum())
    absterm = (np.abs(dr[:, m]) * ft).sum(axis=1).max()
    print(f"ion {i}: |F| {np.abs(E[:, i]).max():.3e} sum|terms| {float(absterm):.3e} dist-from-ball-ctr {rb:.2f} "
          f"dC {d[i]:.2e} |C-X| {float(np.abs(C[:, i] - X).max()):.2e} |E-X| {float(np.abs(E[:, i] - X).max()):.2e}", flush=True)
