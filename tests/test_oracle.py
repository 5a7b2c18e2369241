"""Pin the oracle (CPU restatement of SpeedUp's hot path) before trusting it.

- drand48 stream vs glibc's own srand48/drand48 (the reference's RNG, SpeedUp:1219, :486).
- Philox4x32-10 vs the published Random123 known-answer vectors.
- Yukawa force / pair potential / wrap vs the reference's own compiled MD code and the golden
  vectors it produced (tests/golden/ref_md_n4096.npz, tests/golden/make_golden.py).
- per-ion qstep vs an independent dense numpy transcription (tests/dense_qt.py) — the QT part
  is "parity unpinned" against the reference itself (Armadillo is absent).
"""
import ctypes
import math
import os

import numpy as np
import pytest

from tests import dense_qt

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_md_n4096.npz")


def test_drand48_matches_glibc(orc):
    libc = ctypes.CDLL(None)
    libc.drand48.restype = ctypes.c_double
    for seed in (0, 1, 12346, 2**31 + 7, 2**32 - 1):
        libc.srand48(ctypes.c_long(seed))
        ref = [libc.drand48() for _ in range(2000)]
        mine = orc.drand48_stream(seed, 2000)
        assert np.array_equal(np.array(ref), mine), seed


@pytest.mark.parametrize("ctr,key,expect", [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_kat(orc, ctr, key, expect):
    assert orc.philox4x32_10(ctr, key) == expect


def test_philox_uniform_range_and_independence(orc):
    u = np.array([orc.philox_uniform(12345, 1, i, q, d) for i in range(50) for q in range(4) for d in range(5)])
    assert (u >= 0).all() and (u < 1).all()
    assert len(np.unique(u)) == len(u)
    assert abs(u.mean() - 0.5) < 0.05


def _rel_force_err(F, G):
    return np.abs(F - G).max() / np.abs(G).max()


@pytest.mark.parametrize("case", [0, 1])
def test_oracle_forces_match_reference_golden(orc, case):
    g = np.load(GOLD)
    L, kappa = float(g["L"]), float(g["kappa"])
    F = orc.forces_raw(g[f"R{case}"], L, 1.0 / kappa, nthreads=8)
    A = g[f"A{case}"]
    # same law written differently (pow(r,-3)+kappa/r^2 vs (1/r+1/lDeb)/r^2): ulp-level only
    assert _rel_force_err(F, A) < 1e-13
    # per-component, relative to the sum of |pair terms| scale
    assert np.allclose(F, A, rtol=1e-11, atol=1e-12 * np.abs(A).max())


@pytest.mark.parametrize("case", [0, 1])
def test_oracle_epotential_matches_reference_golden(orc, case):
    g = np.load(GOLD)
    L, kappa = float(g["L"]), float(g["kappa"])
    e = orc.epotential_raw(g[f"R{case}"], L, 1.0 / kappa)   # (1/N) sum_{i<j} u
    ref = g[f"U{case}"].sum() / 2 / 4096
    assert abs(e - ref) <= 1e-12 * abs(ref)


def test_wrap_matches_reference_golden():
    g = np.load(GOLD)
    L = float(g["L"])
    dt = 0.005
    R = g["R0"] + dt * g["V0"] + dt * dt / 2 * g["A0"]
    R = np.where(R < 0, R + L, R)
    R = np.where(R > L, R - L, R)
    assert np.array_equal(R, g["Rstep0"])


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle", "_ref", "libmdref.so")),
                    reason="reference MD build not present")
def test_oracle_forces_match_reference_live(orc):
    L = orc.ref().mdref_L()
    rng = np.random.default_rng(7)
    R = rng.uniform(0, L, (3, 4096))
    A = orc.ref_accelerations(R)
    F = orc.forces_raw(R, L, 2.0, nthreads=8)
    assert _rel_force_err(F, A) < 1e-13


def test_init_reproduces_reference_particle_count(orc):
    # seed 12346 at N0=3500 realises N=3573
    s = orc.OracleSim(N0=3500, seed=12346).init()
    assert s.N == 3573
    st = s.get_state()
    L = s.const("L")
    assert (st["R"] > 0).all() and (st["R"] <= L).all()
    assert (st["V"] == 0).all()
    norm = (st["psi"] ** 2).sum(axis=(1, 2))
    assert np.allclose(norm, 1.0, atol=1e-15)
    assert (st["psi"][:, 2:, :] == 0).all()


def test_derived_constants(orc):
    s = orc.OracleSim(N0=3500)
    assert s.const("plasmaToQuantumTimestepRatio") == 25
    assert s.const("quantumTimestep") == 0.002 / 25
    assert abs(s.const("gamToEinsteinFreq") - 123.0861) < 1e-4
    assert abs(s.const("plasVelToQuantVel") - 1.32686) < 1e-5
    assert abs(s.const("vKick") - 9.10418e-4) < 1e-9
    assert abs(s.const("L") - 24.474785) < 1e-6
    # KAT-1: decayMatrix = (1+r) on the P levels, 0 elsewhere
    for k in range(12):
        d = s.const(f"decay{k}")
        if 2 <= k <= 5:
            assert abs(d - 1.0617) < 1e-15
        else:
            assert d == 0.0


P_DEF = dict(Om=1.0, OmDP=1.0, detuning=-1.0, detuningDP=1.0, fracOfSig=0.0, Te=19.0, density=2.0, sig0=4.0)


def _rand_psi(rng, pops=True):
    z = rng.normal(size=12) + 1j * rng.normal(size=12)
    if not pops:
        z[2:] = 0
    return z / np.linalg.norm(z)


@pytest.mark.parametrize("params", [P_DEF, dict(P_DEF, detuningDP=1.0, detuning=-0.5, Om=0.7, OmDP=1.3),
                                    dict(P_DEF, fracOfSig=0.4)])
def test_qstep_no_jump_matches_dense_transcription(orc, params):
    rng = np.random.default_rng(3)
    s = orc.OracleSim(**{k: v for k, v in params.items()})
    for trial in range(20):
        psi = _rand_psi(rng)
        vx = rng.normal(0, 0.3)
        tp = rng.uniform(0, 0.05)
        t = rng.uniform(0, 5)
        u = [1.0, 0, 0, 0, 0]  # no jump
        res = s.qstep_ion(t, np.stack([psi.real, psi.imag], -1).reshape(-1), vx, tp, u)
        d_psi, d_vx, d_tp, d_j = dense_qt.qstep_ion(psi, vx, tp, t, u, params)
        assert not res["jumped"] and not d_j
        got = res["psi"].reshape(12, 2)
        assert np.abs(got[:, 0] + 1j * got[:, 1] - d_psi).max() < 1e-14
        assert abs(res["vx"] - d_vx) < 1e-17 + 1e-14 * abs(d_vx - vx)
        assert res["tPart"] == d_tp


def test_qstep_jump_branch_matches_dense_transcription(orc):
    rng = np.random.default_rng(5)
    s = orc.OracleSim()
    seen = set()
    for trial in range(400):
        psi = _rand_psi(rng)
        u = [0.0] + list(rng.uniform(size=4))
        res = s.qstep_ion(1.0, np.stack([psi.real, psi.imag], -1).reshape(-1), 0.1, 0.02, u)
        d_psi, d_vx, d_tp, d_j = dense_qt.qstep_ion(psi, 0.1, 0.02, 1.0, u, P_DEF)
        assert res["jumped"] and d_j
        got = res["psi"].reshape(12, 2)
        assert np.array_equal(got[:, 0] + 1j * got[:, 1], d_psi)
        assert res["vx"] == d_vx and res["tPart"] == 0.0
        assert res["ndraws"] in (4, 5)
        seen.add(int(np.argmax(np.abs(d_psi))))
    assert seen == set(range(12)) - {2, 3, 4, 5}   # every S and D target reached


def test_qstep_kat_no_light_is_identity_on_S(orc):
    # Om = OmDP = 0 and psi in the S manifold: dp = 0, H = 0 on S, no kick, psi unchanged.
    s = orc.OracleSim(Om=0.0, OmDP=0.0)
    rng = np.random.default_rng(11)
    for _ in range(5):
        psi = _rand_psi(rng, pops=False)
        res = s.qstep_ion(0.3, np.stack([psi.real, psi.imag], -1).reshape(-1), 0.2, 0.0, [0.5, 0, 0, 0, 0])
        got = res["psi"].reshape(12, 2)
        assert not res["jumped"]
        assert np.allclose(got[:, 0] + 1j * got[:, 1], psi, atol=1e-15, rtol=0)
        assert res["vx"] == 0.2


def test_qstep_kat_single_P_level(orc):
    # Om = OmDP = 0, psi = |P+3/2>: the no-jump branch is an Euler-type step of the *normalized*
    # non-Hermitian evolution (M y / sqrt(1 - dp)), so |psi| stays 1 and the phase advances by
    # -E h with E = -detuning - v_q = 1 (SpeedUp:506, :526-567), both to O(h^2).
    s = orc.OracleSim(Om=0.0, OmDP=0.0)
    psi = np.zeros(24); psi[4] = 1.0
    h = s.const("quantumTimestep") * s.const("gamToEinsteinFreq")
    res = s.qstep_ion(0.0, psi, 0.0, 0.0, [1.0, 0, 0, 0, 0])
    z = res["psi"][4] + 1j * res["psi"][5]
    assert abs(abs(z) - 1.0) < h * h
    assert abs(np.angle(z) - (-1.0 * h)) < h * h
    assert np.all(res["psi"][np.r_[0:4, 6:24]] == 0)


@pytest.mark.parametrize("model,Om,det", [(1, 0.7, -2.5), (2, 2.0, 0.0), (3, 1.3, -1.0)])
def test_pump_qstep_matches_dense_transcription(orc, model, Om, det):
    """optical-pumping qstep (randomFrozenStartTag*.cpp) of the oracle vs the numpy transcription:
    the no-jump RK branch to 1e-14, every jump branch exactly"""
    from tests import dense_pump
    rng = np.random.default_rng(7 + model)
    n = 5 if model == 3 else 7
    s = orc.OracleSim(qt_model=model, Om=Om, detuning=det)
    for trial in range(20):
        z = np.zeros(12, complex)
        z[:n] = rng.normal(size=n) + 1j * rng.normal(size=n)
        z /= np.linalg.norm(z)
        vx = rng.normal(0, 0.3)
        res = s.qstep_ion(0.0, np.stack([z.real, z.imag], -1).reshape(-1), vx, 0.01, [1.0, 0, 0, 0, 0])
        d_psi, d_vx, d_tp, d_j = dense_pump.qstep_ion(z, vx, 0.01, [1.0], model, Om, det)
        assert not res["jumped"] and not d_j
        got = res["psi"].reshape(12, 2)
        assert np.abs(got[:, 0] + 1j * got[:, 1] - d_psi).max() < 1e-14
        assert res["vx"] == vx                       # no optical force in the pumping models
    targets = set()
    for trial in range(600):
        z = np.zeros(12, complex)
        z[:n] = rng.normal(size=n) + 1j * rng.normal(size=n)
        z /= np.linalg.norm(z)
        u = [0.0] + list(rng.uniform(size=4))
        res = s.qstep_ion(0.0, np.stack([z.real, z.imag], -1).reshape(-1), 0.1, 0.02, u)
        d_psi, d_vx, d_tp, d_j = dense_pump.qstep_ion(z, 0.1, 0.02, u, model, Om, det)
        assert res["jumped"] and d_j
        got = res["psi"].reshape(12, 2)
        assert np.array_equal(got[:, 0] + 1j * got[:, 1], d_psi)
        assert res["vx"] == 0.1 and res["tPart"] == 0.0
        targets.add(int(np.argmax(np.abs(d_psi))))
    assert targets == ({0, 1, 4} if model == 3 else {0, 1, 6})


def test_pump_kat_decay_matrix(orc):
    """KAT: the pumping decay matrix sum_j gs[j] cs_j^H cs_j is (1 + r) on every P level for both
    level schemes (408: 1 + r, 2/3 + 1/3 + r, 1/3 + 2/3 + r, 1 + r; 422: 2/3 + 1/3 + r each)"""
    from tests import dense_pump
    for model in (1, 3):
        r = dense_pump.model_constants(model)["decayRatio"]
        n, w, cs, gs = dense_pump.operators(model, r)
        D = sum(gs[j] * cs[j].conj().T @ cs[j] for j in range(len(cs)))
        P = range(2, 6) if model == 1 else range(2, 4)
        for k in range(n):
            assert abs(D[k, k] - ((1 + r) if k in P else 0.)) < 1e-15


@pytest.mark.parametrize("model,density", [(1, 2.0), (2, 2.0), (3, 2.0), (1, 0.5), (3, 3.0), (0, 2.0)])
def test_pump_program_constants(orc, model, density):
    """KAT of the programs' own constants: SpeedUp ceil(34.81/sqrt(d)) (:83); the 408 programs
    round(34.81/sqrt(d)) (randomFrozenStartTag408Linear.cpp:73); the 422 program gamma x .894,
    round(34.81*.894/sqrt(d)), velocity x .967, D/S ratio 0.0754 (randomFrozenStartTag422Linear.cpp
    :66-74, :116).  At density 2: ratios 25, 25, 22."""
    import math
    from tests import dense_pump
    s = orc.OracleSim(qt_model=model, density=density)
    if model == 0:
        assert s.const("plasmaToQuantumTimestepRatio") == math.ceil(34.81 / math.sqrt(density))
        assert s.const("decayRatioD5Halves") == 0.0617
        return
    c = dense_pump.model_constants(model, density)
    assert s.const("plasmaToQuantumTimestepRatio") == c["ratio"]
    assert s.const("plasVelToQuantVel") == c["pv2q"]
    assert s.const("decayRatioD5Halves") == c["decayRatio"]
    if density == 2.0:
        assert c["ratio"] == (22 if model == 3 else 25)


def test_run_layout_and_formats(orc, tmp_path):
    s = orc.OracleSim(N0=60, tmax=0.09, sampleFreq=5, seed=99, job=3, rng_mode=0,
                      saveDirectory=str(tmp_path) + "/")
    assert s.run() == 0
    d = s.save_directory
    assert d.endswith("Ge10Density2000E+11Sig040Te19SigFrac0DetSP-100DetDP100OmSP100OmDP100NumIons60/job3/")
    files = sorted(os.listdir(d))
    c = s.counters()
    N = s.N
    assert f"ions_timestep{c['c0']:06d}.dat" in files
    assert f"conditions_timestep{c['c0']:06d}.dat" in files
    assert f"wvFns_timestep{c['c0']:06d}.dat" in files
    assert sum(f.startswith("VZERO_") for f in files) == 13
    assert "energies.dat" in files
    nout = c["counter"]
    assert nout >= 1
    for k in range(nout):
        for ax in "XYZ":
            assert f"vel_dist{ax}_time{k:06d}.dat" in files
        assert f"statePopulationsVsVTime{k:06d}.dat" in files
    ions = open(os.path.join(d, f"ions_timestep{c['c0']:06d}.dat")).read()
    assert ions == f"{N}\t{nout}"
    lines = open(os.path.join(d, f"conditions_timestep{c['c0']:06d}.dat")).read().splitlines()
    assert len(lines) == N and all(l.endswith("\t") and l.count("\t") == 6 for l in lines)
    e = np.loadtxt(os.path.join(d, "energies.dat"), ndmin=2)
    assert e.shape == (nout, 7)


def test_resume_roundtrip(orc, tmp_path):
    s = orc.OracleSim(N0=60, tmax=0.05, sampleFreq=1000, seed=5, job=1, saveDirectory=str(tmp_path) + "/")
    assert s.run() == 0
    c0 = s.counters()["c0"]
    st = s.get_state()
    r = orc.OracleSim(N0=60, tmax=0.05, newRun=0, c0=c0, saveDirectory=str(tmp_path) + "/")
    r.setup_directories()
    assert r.read_conditions(c0) == 0
    st2 = r.get_state()
    assert r.N == s.N
    assert np.allclose(st2["R"], st["R"], rtol=1e-5, atol=1e-6)   # %lg = 6 significant digits
    assert np.allclose(st2["psi"], st["psi"], rtol=1e-5, atol=1e-6)
    assert r.t == (c0 - 9.0) * 0.002 + 0.02                        # SpeedUp:789
    assert (st2["tPart"] == 0).all()                                # not restored (App. C-8)


def test_forces_row_partition_invariance(orc):
    rng = np.random.default_rng(2)
    L = 12.79
    R = rng.uniform(0, L, (3, 501))
    F = orc.forces_raw(R, L, 1.8257)
    G = np.zeros_like(F)
    for lo, hi in ((0, 100), (100, 377), (377, 501)):
        G[:, lo:hi] = orc.forces_rows(R, lo, hi, L, 1.8257)[:, lo:hi]
    assert np.array_equal(F, G)


def test_philox_mode_thread_invariance(orc):
    a = orc.OracleSim(N0=300, seed=8, rng_mode=1, nthreads=1).init()
    b = orc.OracleSim(N0=300, seed=8, rng_mode=1, nthreads=4).init()
    a.md_steps(2); b.md_steps(2)
    sa, sb = a.get_state(), b.get_state()
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(sa[k], sb[k])
