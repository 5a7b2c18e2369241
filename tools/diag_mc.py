"""Lock-step MC of the engine (force_kernel 1) and the reference: first divergence."""
import os, sys, tempfile
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdqtplasmasims_amd import mdmc
from oracle import oracle as O

tmp = tempfile.mkdtemp()
fk = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ref = O.RefMCMD(seed=12, save_directory=tmp + "/")
eng = mdmc.MonteCarloMD(seed=12, saveDirectory=tmp + "/", force_kernel=fk)
ref.init(); eng.init()
R0, _, _, U0 = ref.get_state(); R1, _, _, U1 = eng.get_state()
print("init U rel", np.abs(U1 - U0).max() / np.abs(U0).max(), flush=True)
for k in range(3000):
    ref.monte_carlo(1); a = eng.monte_carlo(1)
    R0, _, _, U0 = ref.get_state(); R1, _, _, U1 = eng.get_state()
    if not np.array_equal(R0, R1):
        d = np.argwhere(R0 != R1)
        print("step", k, "accepted(eng)", a, "differing", d[:6].tolist(), "dR", np.abs(R0 - R1).max(), flush=True)
        p = d[0][1]
        print("ref R[p]", R0[:, p], "eng R[p]", R1[:, p])
        print("U rel", np.abs(U1 - U0).max() / np.abs(U0).max(), "sumU", U0.sum(), U1.sum())
        break
    if k % 500 == 0:
        print(k, "U rel", np.abs(U1 - U0).max() / np.abs(U0).max(), flush=True)
else:
    print("no divergence in 3000 steps")
