"""Generate the golden vectors under tests/golden/ from the reference's OWN compiled code.

The reference's MD-only program /root/reference/MonteCarloFollowedByMDAndTempAnisotropy.cpp is
built unmodified by oracle/ref/Makefile into oracle/_ref/libmdref.so (its N = 4096, kappa = 0.5,
L = (4096*4pi/3)^(1/3) are fixed by that file).  For seeded synthetic positions this script
records what the reference computes:
  A   = calculateAccelerations()                 (:387-448)  Yukawa force, minimum image, cutoff
  U   = calculatePotentialEnergyForParticles()   (:207-244)  per-particle pair-potential sums
  R1  = stepPositions()                          (:453-467)  position update + periodic wrap
Run:  python tests/golden/make_golden.py        (needs /root/reference; output is committed)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


def main():
    O.build()
    L = O.ref().mdref_L()
    rng = np.random.default_rng(20261015)
    out = {}
    # case 0: uniform random positions in (0, L]^3
    R0 = rng.uniform(0, L, (3, 4096))
    # case 1: clustered positions straddling the periodic boundary + near-cutoff separations
    c = rng.normal(0, 0.15 * L, (3, 4096)) % L
    c[:, :64] = np.array([[0.01], [0.01], [0.01]]) + rng.uniform(0, 0.02, (3, 64))
    c[:, 64:128] = np.array([[L - 0.01], [L - 0.01], [L - 0.01]]) - rng.uniform(0, 0.02, (3, 64))
    c[0, 128:192] = (c[0, 0:64] + L / 2 * (1 - 1e-9)) % L
    c[1:, 128:192] = c[1:, 0:64]
    R1c = c
    V0 = rng.normal(0, 0.6, (3, 4096))
    for k, R in enumerate((R0, R1c)):
        out[f"R{k}"] = R
        out[f"A{k}"] = O.ref_accelerations(R)
        out[f"U{k}"] = O.ref_particle_potentials(R)
    out["V0"] = V0
    out["Rstep0"] = O.ref_step_positions(R0, V0, out["A0"])
    out["L"] = np.array(L)
    out["kappa"] = np.array(O.ref().mdref_kappa())
    np.savez_compressed(os.path.join(HERE, "ref_md_n4096.npz"), **out)
    print("wrote", os.path.join(HERE, "ref_md_n4096.npz"))


if __name__ == "__main__":
    main()
