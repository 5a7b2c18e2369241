"""The production RNG against the reference's own random-number order, as ensembles (BASELINE.md §3:
long runs agree "within statistical error").

The device path draws its quantum-jump uniforms from Philox keyed by (seed, job, ion, qstep)
(rng_mode 1) where SpeedUp draws from one shared drand48 stream in ion order (SpeedUp:486,
:575-591, seeded :1219; rng_mode 0 reproduces that order exactly, tests/test_gpu_parity.py).  The
two streams give different trajectories, so the check is statistical: 32 seeds x 200 MD steps at
N0 = 500 with QT on, each seed run in both modes from the same init() (same drand48 positions and
wavefunctions), and the observables the reference writes — EkinX of energies.dat (:939-955) and
the P-state population of statePopulationsVsVTime (:1010-1024) — compared at 5 sample times.
Paired differences (same seed, same initial state): |mean(d)| <= 3 sigma_d / sqrt(32).  The seeds
are fixed, so the test is deterministic."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEEDS = range(101, 133)
SAMPLE_MD_STEPS = (40, 80, 120, 160, 200)


def _observables(st):
    V, psi = st["V"], st["psi"]
    vx = V[0]
    ekx = 0.5 * ((vx - vx.mean()) ** 2).mean()                      # EkinX (SpeedUp:939-947)
    pop_p = (psi[:, 2:6, :] ** 2).sum(axis=(1, 2)).mean()           # P levels 2..5 (App. A)
    return ekx, pop_p


def _trajectory(M, seed, rng_mode):
    s = M.Simulation(N0=500, seed=seed, job=1, rng_mode=rng_mode).init()
    out, done = [], 0
    for k in SAMPLE_MD_STEPS:
        s.md_steps(k - done)
        done = k
        out.append(_observables(s.get_state()))
    njump = int((s.get_state()["tPart"] < done * 0.002 - 1e-9).sum())
    s.close()
    return np.array(out), njump


def test_philox_ensemble_matches_reference_drand48_order():
    import mdqtplasmasims_amd as M
    if M.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked tests")
    A, B, jumps = [], [], 0
    for seed in SEEDS:
        a, ja = _trajectory(M, seed, 1)           # Philox (production)
        b, jb = _trajectory(M, seed, 0)           # the reference's drand48 order
        A.append(a); B.append(b)
        jumps += ja + jb
    A, B = np.array(A), np.array(B)               # [seed][time][observable]
    n = len(SEEDS)
    d = A - B
    z = np.abs(d.mean(axis=0)) / (d.std(axis=0, ddof=1) / np.sqrt(n))
    for t, k in enumerate(SAMPLE_MD_STEPS):
        print(f"MD step {k}: EkinX philox {A[:, t, 0].mean():.6e} drand48 {B[:, t, 0].mean():.6e} z={z[t, 0]:.2f}; "
              f"P pop philox {A[:, t, 1].mean():.6e} drand48 {B[:, t, 1].mean():.6e} z={z[t, 1]:.2f}")
    assert jumps > 1000                            # the two streams really decided many jumps
    assert np.all(d.std(axis=0) > 0)               # the streams differ (not the same draws)
    assert np.all(z <= 3.0), z
