"""GPU parity across the reference's user inputs.

SpeedUp:58-74 lists the parameters "you'll ever really want to change".  The other GPU tests run
density 2 (substep ratio 25), fracOfSig 0, no renormalisation and detuning -1; here each case
changes one of them and runs 3 MD steps through the C ABI against the oracle (oracle/mdqt_oracle.c,
a line-cited restatement of SpeedUp; parity of the QT arithmetic is unpinned against the reference
binary, which needs Armadillo — DESIGN.md §4), in both RNG modes:

  * rng_mode 1 (Philox, the production stream): same jump set, |dR|, |dV| <= 1e-10, |dpsi| <= 1e-9
    (the gates of test_md_steps_short_horizon);
  * rng_mode 0 (the reference's drand48 order): the same, plus the same stream position.

Each case asserts which substep kernel instance its production launch (the last one) took
(mdqt_internal.hpp QTKernel), so that the non-default instances are the code under test:

  density 0.5 / 1.0 / 3.0   ratio ceil(34.81 / sqrt(density)) = 50 / 35 / 21 (:83): the first two
                            exceed MAXSUB = 32, so every MD interval is two launches (32 + 18,
                            32 + 3), the second summing F itself (nseg 1)
  fracOfSig 0.4             expDetuning(t) != 0 (:447, :506-510): the non-EDZ instance
                            k_substeps_lanes_im<true, false>; once with the default Te / sig0 and
                            once with Te 5, sig0 2
  reNormalizewvFns 1        :706-712: k_substeps_lanes_im<true, true, false>
  detuning -2               :70 (the S-P diagonal)
  Ge 0.5                    :60 (kappa = sqrt(1.5): the force law's screening length)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

QTK_LANES_IM_EDZ = 1          # k_substeps_lanes_im<true, true, true> (production, no renorm, e(t) = 0)
QTK_LANES_IM = 2              # k_substeps_lanes_im<true, false> (e(t) != 0)
QTK_LANES_IM_EDZ_RN = 7       # k_substeps_lanes_im<true, true, false> (reNormalizewvFns)

CASES = [
    ("density0.5", dict(density=0.5), 50, QTK_LANES_IM_EDZ),
    ("density1", dict(density=1.0), 35, QTK_LANES_IM_EDZ),
    ("density3", dict(density=3.0), 21, QTK_LANES_IM_EDZ),
    ("fracOfSig0.4", dict(fracOfSig=0.4), 25, QTK_LANES_IM),
    ("fracOfSig0.4_Te5_sig02", dict(fracOfSig=0.4, Te=5.0, sig0=2.0), 25, QTK_LANES_IM),
    ("renorm", dict(reNormalizewvFns=1), 25, QTK_LANES_IM_EDZ_RN),
    ("detuning-2", dict(detuning=-2.0), 25, QTK_LANES_IM_EDZ),
    ("Ge0.5", dict(Ge=0.5), 25, QTK_LANES_IM_EDZ),
]


@pytest.fixture(scope="module")
def eng():
    import mdqtplasmasims_amd as M
    if M.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked tests")
    return M


@pytest.mark.parametrize("rng_mode", [1, 0])
@pytest.mark.parametrize("name,extra,ratio,inst", CASES, ids=[c[0] for c in CASES])
def test_user_input_md_steps_match_oracle(eng, orc, name, extra, ratio, inst, rng_mode):
    kw = dict(N0=500, seed=12346, job=1, rng_mode=rng_mode, **extra)
    s = eng.Simulation(**kw).init()
    o = orc.OracleSim(nthreads=8 if rng_mode == 1 else 1, **kw).init()
    assert s.N == o.N
    assert int(s.const("plasmaToQuantumTimestepRatio")) == int(o.const("plasmaToQuantumTimestepRatio")) == ratio
    if rng_mode == 0:
        assert s.drand48_state == orc.lib().orc_get_drand48_state(o.h)
    s.md_steps(3); o.md_steps(3)
    # the last launch of the third MD interval (t > 0 throughout): the instance this input selects
    assert s.const("qt_kernel") == inst, (name, s.const("qt_kernel"))
    if ratio > 32:
        assert s.const("qt_kernel_nseg") == 1          # the interval's second launch sums F itself
    a, b = s.get_state(), o.get_state()
    assert a["t"] == b["t"] and s.qstep_index == o.qstep_index == 3 * ratio
    if rng_mode == 0:
        assert s.drand48_state == orc.lib().orc_get_drand48_state(o.h)   # same number of draws
    jumped = b["tPart"] < 3 * ratio * o.const("quantumTimestep") - 1e-12
    assert np.array_equal(a["tPart"] < 3 * ratio * o.const("quantumTimestep") - 1e-12, jumped)
    assert np.array_equal(a["tPart"] == 0, b["tPart"] == 0)
    dR, dV = np.abs(a["R"] - b["R"]).max(), np.abs(a["V"] - b["V"]).max()
    dpsi = np.abs(a["psi"] - b["psi"]).max()
    print(f"{name} rng_mode {rng_mode}: N={s.N} ratio={ratio} jumps={int(jumped.sum())} |dR|={dR:.2e} "
          f"|dV|={dV:.2e} |dpsi|={dpsi:.2e}")
    assert dR <= 1e-10 and dV <= 1e-10
    assert dpsi <= 1e-9
    if extra.get("reNormalizewvFns"):
        nrm = (a["psi"] ** 2).sum(axis=(1, 2))
        assert np.abs(nrm - 1).max() < 1e-12           # :706-712 renormalised every qstep
    s.close(); o.close()


def test_fracofsig_expdetuning_enters_the_phase(eng, orc):
    """expDetuning (:447) is not a no-op: fracOfSig 0.4 and 0 give different wavefunctions after one
    MD step (guards the non-EDZ case above against testing a zero term)"""
    out = []
    for f in (0.0, 0.4):
        s = eng.Simulation(N0=300, seed=12346, fracOfSig=f).init()
        s.md_steps(2)
        out.append(s.get_state()["psi"])
        s.close()
    assert np.abs(out[0] - out[1]).max() > 1e-8


def test_run_files_at_density_1_match_oracle(eng, orc, tmp_path):
    """mdqt_run() (SpeedUp main() loop) at density 1 — ratio 35, two launches per MD interval — against
    OracleSim.run(): the same files, equal to the printed %lg precision"""
    kw = dict(N0=60, tmax=0.09, sampleFreq=5, seed=99, job=3, rng_mode=1, density=1.0)
    s = eng.Simulation(saveDirectory=str(tmp_path / "gpu") + "/", **kw)
    s.run()
    o = orc.OracleSim(saveDirectory=str(tmp_path / "cpu") + "/", **kw)
    assert o.run() == 0
    import os
    A = {f: open(os.path.join(s.save_directory, f)).read() for f in sorted(os.listdir(s.save_directory))}
    B = {f: open(os.path.join(o.save_directory, f)).read() for f in sorted(os.listdir(o.save_directory))}
    assert "Density1000E+11" in s.save_directory
    assert sorted(A) == sorted(B) and len(A) > 5
    assert s.counters()["c0"] == o.counters()["c0"] and s.counters()["counter"] == o.counters()["counter"]
    for f in A:
        a, b = A[f], B[f]
        if f.startswith("ions_"):
            assert a == b
            continue
        la, lb = a.splitlines(), b.splitlines()
        assert len(la) == len(lb), f
        xa = np.array([[float(v) for v in l.split()] for l in la if l.strip()])
        xb = np.array([[float(v) for v in l.split()] for l in lb if l.strip()])
        assert xa.shape == xb.shape, f
        assert np.allclose(xa, xb, rtol=2e-5, atol=1e-9 * max(1.0, np.abs(xb).max())), f
