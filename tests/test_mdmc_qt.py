"""The QT spin-tagging variants of the MC + MD program (include/mdmc.h, qt_model 1..3):
MonteCarloFollowedByQTTagging408Linear.cpp / 408Quad.cpp / 422Linear.cpp ("QTT").

These programs need Armadillo (absent here), so they are not built; the oracle is the C
restatement of the pumping qstep (oracle/mdqt_oracle.c: qstep_ion_pump, pinned to the dense
transcription tests/dense_pump.py) run with the QTT constants, the Python drand48 / Philox
restatements, and numpy for the tagged-ion observables.  The MC / MD stages are the MCMD engine's
(tests/test_mdmc.py pins them to the reference build).

Tolerances: wavefunction init bit for bit (drand48 default stream, the reference's operations);
one QT step <= 1e-12 (the reassociated QT kernel vs the oracle's exact operations); tags exact;
moments <= 1e-12 relative; velocity distributions <= 1e-12 of the largest bin (exp ulps, sum order).
"""
import math
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MODELS = [1, 2, 3]


@pytest.fixture(scope="module")
def mc():
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd import mdmc
    if M.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked tests")
    return mdmc


def qtt_constants(model, n=2.0, timeStep=0.005, tpumpreal=None):
    """QTT408Linear.cpp:115-121 / 408Quad.cpp:110-120 / 422Linear.cpp:115-121 (C round: half away)"""
    if model == 3:
        gamToE = 174.07 * .894 / math.sqrt(n)
        ratio = int(math.floor(87 * .894 / math.sqrt(n) + 0.5))
        pv2q = 1.1821 * n ** (1.0 / 6) * .967
        r = 0.0753
    else:
        gamToE = 174.07 / math.sqrt(n)
        ratio = int(math.floor(87 / math.sqrt(n) + 0.5))
        pv2q = 1.1821 * n ** (1.0 / 6)
        r = 0.0617
    out = dict(gamToE=gamToE, ratio=ratio, dtQ=timeStep / ratio, pv2q=pv2q, r=r)
    if tpumpreal is not None:
        out["pump"] = int(math.floor(tpumpreal * 813490 * math.sqrt(n) / timeStep + 0.5))
    return out


@pytest.mark.parametrize("model", MODELS)
def test_qtt_constants(mc, model):
    e = mc.MonteCarloMD(qt_model=model, N=512)
    c = qtt_constants(model, tpumpreal=e.p.tpumpreal)
    assert e.const("plasmaToQuantumTimestepRatio") == c["ratio"]
    assert e.const("quantumTimestep") == c["dtQ"]
    assert e.const("gamToEinsteinFreq") == c["gamToE"]
    assert e.const("plasVelToQuantVel") == c["pv2q"]
    assert e.const("decayRatio") == c["r"]
    assert e.const("pumpMDTimeSteps") == c["pump"]
    assert (model, c["ratio"]) in ((1, 62), (2, 62), (3, 55))
    e.close()


def test_qtt_init_wavefunctions(mc, orc):
    """QTT:224-239 with drand48's default state (the programs never call srand48)"""
    e = mc.MonteCarloMD(qt_model=1, N=512, seed=5)
    e.init()
    psi = e.get_psi()
    u = orc.drand48_stream(0x1234ABCD, 4 * 512).reshape(512, 4)
    r1, r2, r3, r4 = u.T
    sign = np.where(r3 < 0.5, -1.0, 1.0)
    sign2 = np.where(r4 < 0.5, -1.0, 1.0)
    assert np.array_equal(psi[:, 0].real, np.sqrt(r1)) and np.all(psi[:, 0].imag == 0)
    assert np.array_equal(psi[:, 1].real, sign2 * np.sqrt(1 - r1) * np.sqrt(r2))
    assert np.array_equal(psi[:, 1].imag, sign * np.sqrt(1 - r1) * np.sqrt(1 - r2))
    assert np.all(psi[:, 2:] == 0)
    e.close()


@pytest.mark.parametrize("model", MODELS)
def test_qtt_qstep_matches_oracle(mc, orc, model):
    """one pump qstep of every ion vs the oracle's pumping qstep with the QTT constants and the
    same Philox draws (seed, job, ion, qstep 0, draws 0..4)"""
    seed, job = 21, 2
    e = mc.MonteCarloMD(qt_model=model, N=512, seed=seed, job=job)
    e.init()
    rng = np.random.default_rng(model)
    n = 5 if model == 3 else 7
    z = np.zeros((512, 12), complex)
    z[:, :n] = rng.normal(size=(512, n)) + 1j * rng.normal(size=(512, n))
    z /= np.linalg.norm(z, axis=1, keepdims=True)
    z[:40, 2:2 + (2 if model == 3 else 4)] *= 30.0            # heavy P populations: jumps
    z /= np.linalg.norm(z, axis=1, keepdims=True)
    e.set_psi(z)
    _, V, _, _ = e.get_state()
    e.qsteps(1)
    got = e.get_psi()
    _, V1, _, _ = e.get_state()
    assert np.array_equal(V1, V)                                 # no kick in the pumping models
    c = qtt_constants(model)
    o = orc.OracleSim(qt_model=model, Om=e.p.Om, detuning=e.p.detuning, density=2.0)
    o.set_qt_constants(c["dtQ"], c["gamToE"], c["pv2q"], c["r"])
    jumps = 0
    for i in range(512):
        u = [orc.philox_uniform(seed, job, i, 0, d) for d in range(5)]
        res = o.qstep_ion(0.0, np.stack([z[i].real, z[i].imag], -1).reshape(-1), V[0, i], 0.0, u)
        ref = res["psi"].reshape(12, 2)
        ref = ref[:, 0] + 1j * ref[:, 1]
        jumps += res["jumped"]
        assert np.abs(got[i] - ref).max() <= 1e-12, (i, res["jumped"])
    assert jumps > 0
    o.close()
    e.close()


@pytest.mark.parametrize("model", MODELS)
def test_qtt_tags_moments_and_distributions(mc, orc, model):
    seed, job = 8, 1
    e = mc.MonteCarloMD(qt_model=model, N=512, seed=seed, job=job)
    e.init()
    e.qsteps(7)
    psi = e.get_psi()
    tags, cnt = e.tag_qt()
    nr = np.abs(psi) ** 2
    exp = np.zeros(512, np.int32)
    for i in range(512):                                         # QTT:1022-1067 / 422 :992-1034
        rnd = orc.philox_uniform(seed, job, i, 7, 6)
        r2 = orc.philox_uniform(seed, job, i, 7, 7)
        if model == 3:
            up = rnd < nr[i, 0] or (rnd < nr[i, 0] + nr[i, 2] and r2 < 1 / 3) or \
                (nr[i, 0] + nr[i, 2] <= rnd < nr[i, 0] + nr[i, 2] + nr[i, 3] and r2 < 2 / 3)
        else:
            a = nr[i, 0] + nr[i, 2]
            up = rnd < a or (a <= rnd < a + nr[i, 3] and r2 < 2 / 3) or \
                (a + nr[i, 3] <= rnd < a + nr[i, 3] + nr[i, 4] and r2 < 1 / 3)
        exp[i] = up
    assert np.array_equal(tags, exp) and cnt == exp.sum()
    mom, dist = e.tagged_moments_qt()
    _, V, _, _ = e.get_state()
    vx = V[0][tags == 1]
    ref = [vx.sum() / cnt, (vx * vx).sum() / cnt, (vx * vx * vx).sum() / cnt, (vx * vx * vx * vx).sum() / cnt]
    np.testing.assert_allclose(mom, ref, rtol=1e-12, atol=1e-15)
    vel = (np.arange(4001) - 2000) * 0.0025
    V2 = 1. / (2. * 0.002 * 0.002)
    for c in range(3):
        v = V[c][tags == 1]
        P = np.exp(-V2 * (vel[:, None] - v[None, :]) ** 2).sum(1) / (6.0 * math.sqrt(2 * math.pi * 0.002 * 0.002))
        assert np.abs(dist[c] - P).max() <= 1e-12 * P.max()
    e.close()


def test_qtt_run_writes_the_reference_files(mc):
    """QTT main() at reduced sizes: directory name and every file, with its row counts"""
    with tempfile.TemporaryDirectory() as tmp:
        e = mc.MonteCarloMD(qt_model=1, N=512, monteCarloSteps=20000, numPreRecordMDSteps=20,
                            numVelAutoCorrsSteps=40, job=4, saveDirectory=tmp + "/", seed=3)
        e.run()
        d = os.path.join(tmp, "Gamma300Kappa50NumIons512PumpTime200Det250Om70Density20", "job4")
        assert os.path.isdir(d), os.listdir(tmp)
        m = np.loadtxt(os.path.join(d, "taggedMoments.dat"), ndmin=2)
        assert m.shape == (40, 5) and np.isfinite(m).all()
        for k in (0, 39):
            v = np.loadtxt(os.path.join(d, f"vel_distX_timestep{k:06d}.dat"), ndmin=2)
            assert v.shape == (4001, 2) and abs(v[2000, 0]) < 1e-12
        assert np.loadtxt(os.path.join(d, "temperature.dat"), ndmin=2).shape == (40, 1)
        for f in ("VAF", "longViscAutoCorr", "vCubeAutoCorr", "vFourthAutoCorr"):
            assert np.loadtxt(os.path.join(d, f + ".dat"), ndmin=2).shape == (40, 2)
        for k in (0, 10000):
            assert os.path.exists(os.path.join(d, f"pairPairCorrStepNum{k}.dat"))
        e.close()
