import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import mdqtplasmasims_amd as M
from oracle import oracle as O
from tests.test_gpu_large import sample_ions, CONFIGS
s = M.Simulation(seed=12346, job=1, rng_mode=1, **CONFIGS[sys.argv[1]]).init()
N = s.N; L, lDeb = s.const("L"), s.const("lDeb")
R = s.get_state()["R"]
idx = sample_ions(N, 640, np.random.default_rng(11))
G = O.forces_index(R, idx, L, lDeb, nthreads=16)
for mode in (0, 1):
    s.set_option("force_sort", mode); s.forces(); F = s.get_state()["F"]
    err = np.abs(F[:, idx] - G).max() / np.abs(G).max()
    mom = np.abs(F.sum(axis=1)).max() / (np.abs(F).sum() / N)
    print(sys.argv[1], "sort", mode, f"err {err:.3e} mom {mom:.3e}", flush=True)
