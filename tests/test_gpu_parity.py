"""GPU parity of the HIP path (through the C ABI) against the oracle and the reference goldens.

Tolerances (written per test) follow BASELINE.md's parity gates:
  forces <= 1e-13 relative (max-norm), single qstep <= 1e-12, short-horizon energies and velocity
  distributions <= 1e-6 relative.  Pure +,*,/ arithmetic (integrator, init) is compared bit for bit;
  libm differences (exp/sin/cos: ROCm ocml vs glibc, <= 1 ulp) are what the tolerances absorb.
The device path runs the Philox stream (rng_mode=1); the oracle is run in the same mode.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_md_n4096.npz")


@pytest.fixture(scope="module")
def eng():
    import mdqtplasmasims_amd as M
    if M.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked tests")
    return M


def rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


# ---------------------------------------------------------------------------------------------
# kernel 1 vs the reference's own compiled force / potential (golden vectors)
# ---------------------------------------------------------------------------------------------

@pytest.mark.parametrize("case", [0, 1])
@pytest.mark.parametrize("nseg", [1, 0, 7])
@pytest.mark.parametrize("variant", [0, 1])
def test_forces_match_reference_golden(eng, case, nseg, variant):
    from mdqtplasmasims_amd.engine import forces_raw
    g = np.load(GOLD)
    L, kappa = float(g["L"]), float(g["kappa"])
    F = forces_raw(g[f"R{case}"], L, 1.0 / kappa, nseg=nseg, variant=variant)
    A = g[f"A{case}"]
    assert rel(F, A) < 1e-13
    assert np.allclose(F, A, rtol=1e-11, atol=1e-12 * np.abs(A).max())


@pytest.mark.parametrize("case", [0, 1])
@pytest.mark.parametrize("variant", [0, 1])
def test_potentials_match_reference_golden(eng, case, variant):
    from mdqtplasmasims_amd.engine import potentials_raw
    g = np.load(GOLD)
    U = potentials_raw(g[f"R{case}"], float(g["L"]), 1.0 / float(g["kappa"]), variant=variant)
    assert rel(U, g[f"U{case}"]) < 1e-13


def test_forces_match_oracle_bitwise_order(eng, orc):
    """one j-segment = the reference's ascending-j order: only exp ulps may differ"""
    from mdqtplasmasims_amd.engine import forces_raw
    rng = np.random.default_rng(4)
    L = 12.794389
    R = rng.uniform(0, L, (3, 777))
    F = forces_raw(R, L, 1.8257418583505538, nseg=1, variant=0)
    O = orc.forces_raw(R, L, 1.8257418583505538)
    assert rel(F, O) < 1e-14
    # boundary-straddling pairs: exercise the exact minimum-image thresholds at |dx| ~ L/2
    R2 = R.copy()
    R2[:, 1::2] = (R2[:, 0::2][:, :R2[:, 1::2].shape[1]] + L / 2) % L
    F2 = forces_raw(R2, L, 1.8257418583505538, nseg=1, variant=0)
    O2 = orc.forces_raw(R2, L, 1.8257418583505538)
    assert rel(F2, O2) < 1e-14


# ---------------------------------------------------------------------------------------------
# simulation state: init, step, qstep, md steps vs the oracle
# ---------------------------------------------------------------------------------------------

def pair(eng, orc, **kw):
    kw.setdefault("rng_mode", 1)
    s = eng.Simulation(**kw).init()
    o = orc.OracleSim(**kw).init()
    return s, o


@pytest.mark.parametrize("N0", [60, 500, 3500])
def test_init_matches_oracle_bitwise(eng, orc, N0):
    s, o = pair(eng, orc, N0=N0, seed=12346)
    assert s.N == o.N
    a, b = s.get_state(), o.get_state()
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(a[k], b[k]), k
    if N0 == 3500:
        assert s.N == 3573
    ca, cb = s.counters(), o.counters()
    assert ca["c0"] == cb["c0"] == -1
    assert abs(ca["Epot0"] - cb["Epot0"]) <= 1e-12 * abs(cb["Epot0"])


@pytest.mark.parametrize("scheme,variant", [(1, 0), (1, 1), (2, 0), (2, 1), (3, 0), (3, 1)])
def test_forces_match_oracle_after_init(eng, orc, scheme, variant):
    """both force schemes (owner-computes rows; Newton-3 tile pairs) x both pair variants"""
    s, o = pair(eng, orc, N0=3500, seed=12346)
    s.set_option("force_scheme", scheme)
    s.set_option("force_kernel", variant)
    assert s.const("force_scheme") == scheme
    s.forces(); o.forces()
    F, G = s.get_state()["F"], o.get_state()["F"]
    assert rel(F, G) < 1e-13
    assert np.abs(F.sum(axis=1)).max() < 1e-11 * np.abs(F).sum() / F.shape[1]


@pytest.mark.parametrize("N0", [128, 200, 777])
def test_newton3_tiles_ragged_sizes(eng, orc, N0):
    """Newton-3 tile pairs with a partial last tile, diagonal half-steps, substep fusion of slots"""
    s, o = pair(eng, orc, N0=N0, seed=17)
    s.set_option("force_scheme", 2)
    s.forces(); o.forces()
    assert rel(s.get_state()["F"], o.get_state()["F"]) < 1e-13
    s2 = eng.Simulation(N0=N0, seed=17).init()
    s2.set_option("force_scheme", 2)
    s2.md_steps(2)
    o.md_steps(2)
    assert np.abs(s2.get_state()["V"] - o.get_state()["V"]).max() < 1e-10


@pytest.mark.parametrize("N0", [200, 1100, 2500, 5000])
def test_newton3_blocks_sizes(eng, orc, N0):
    """Newton-3 block pairs (half shell of 16-tile blocks): one block, even and odd block counts,
    ragged last tile; then two MD steps"""
    s, o = pair(eng, orc, N0=N0, seed=23)
    s.set_option("force_scheme", 3)
    assert s.const("force_scheme") == 3
    s.forces(); o.forces()
    assert rel(s.get_state()["F"], o.get_state()["F"]) < 1e-13
    s2 = eng.Simulation(N0=N0, seed=23).init()
    s2.set_option("force_scheme", 3)
    s2.md_steps(2)
    o.md_steps(2)
    assert np.abs(s2.get_state()["V"] - o.get_state()["V"]).max() < 1e-10


@pytest.mark.parametrize("world,N0", [(2, 5000), (3, 5000), (2, 400), (3, 700)])
def test_sharded_newton3_blocks_local_group(eng, orc, world, N0):
    """sharded Newton-3 block pairs: every rank computes its blocks' pairs for all ions, the dense
    partials are reduce-scattered (in-process group: summed in rank order) — forces within the
    1e-13 gate of the oracle, trajectories within the short-horizon gate.  N0 = 400 (one block) at
    world 2 and N0 = 700 (two blocks) at world 3 leave a rank without blocks: its dense partial must
    be 0, whatever its unused plan memory holds (the per-J-tile masks)"""
    from mdqtplasmasims_amd.engine import comm_init_local
    kw = dict(N0=N0, seed=9)
    o = orc.OracleSim(nthreads=8, rng_mode=1, **kw).init()
    st = o.get_state()
    sims = [eng.Simulation(world_size=world, rank=r, **kw) for r in range(world)]
    for s in sims:
        s.set_option("force_scheme", 3)
        s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    comm_init_local(sims)
    for s in sims:
        s.allgather_positions()
    for s in sims:
        s.forces()
    o.forces()
    G = o.get_state()["F"]
    for s in sims:
        lo, hi = s.slab_bounds()
        F = s.get_state()["F"][:, lo:hi]
        assert rel(F, G[:, lo:hi]) < 1e-13
    for _ in range(2):
        for s in sims:
            s.substeps(25)
        for s in sims:
            s.allgather_positions()
        for s in sims:
            s.forces()
    for s in sims:
        s.substeps(25)
    o.substeps(25)
    o.md_steps(2)
    b = o.get_state()
    for s in sims:
        lo, hi = s.slab_bounds()
        a = s.get_state()
        assert np.abs(a["R"][:, lo:hi] - b["R"][:, lo:hi]).max() < 1e-10
        assert np.abs(a["V"][:, lo:hi] - b["V"][:, lo:hi]).max() < 1e-10


@pytest.mark.parametrize("t0", [0.0, 0.5])
def test_step_matches_oracle_bitwise(eng, orc, t0):
    """step() = step_R(dt/2); step_V(dt); step_R(dt/2) incl. the t==0 branch and the wrap"""
    s, o = pair(eng, orc, N0=500, seed=3)
    rng = np.random.default_rng(9)
    st = o.get_state()
    V = rng.normal(0, 40.0, st["V"].shape)          # large velocities: many wraps
    F = rng.normal(0, 50.0, st["V"].shape)
    for x in (s, o):
        x.set_state(st["R"], V, st["psi"], st["tPart"], t0)
        x.set_forces(F)
        x.step()
    a, b = s.get_state(), o.get_state()
    assert np.array_equal(a["R"], b["R"])
    assert np.array_equal(a["V"], b["V"])
    assert a["t"] == b["t"] == t0


def _evolved_state(orc, N0=300, seed=21, nmd=4):
    o = orc.OracleSim(N0=N0, seed=seed, rng_mode=1, nthreads=4).init()
    o.md_steps(nmd)
    return o


@pytest.mark.parametrize("qt_math", [0, 1, 2])
def test_qstep_matches_oracle(eng, orc, qt_math):
    o = _evolved_state(orc)
    st = o.get_state()
    s = eng.Simulation(N0=300, seed=21, rng_mode=1)
    s.set_option("qt_math", qt_math)
    s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    s.set_forces(st["F"])
    s.qstep_index = o.qstep_index
    s.qstep(); o.qstep()
    a, b = s.get_state(), o.get_state()
    assert np.abs(a["psi"] - b["psi"]).max() < 1e-12
    assert np.abs(a["V"] - b["V"]).max() < 1e-15
    assert np.array_equal(a["tPart"], b["tPart"])
    assert a["t"] == b["t"] and s.qstep_index == o.qstep_index


def test_qstep_jump_branch_exercised(eng, orc):
    """ions with large P population jump with probability ~dp: force many jumps and compare"""
    o = _evolved_state(orc, nmd=1)
    st = o.get_state()
    psi = np.zeros_like(st["psi"])
    rng = np.random.default_rng(1)
    z = rng.normal(size=(psi.shape[0], 12)) + 1j * rng.normal(size=(psi.shape[0], 12))
    z /= np.linalg.norm(z, axis=1, keepdims=True)
    psi[:, :, 0], psi[:, :, 1] = z.real, z.imag
    s = eng.Simulation(N0=300, seed=21, rng_mode=1, Om=3.0, OmDP=2.0)
    o2 = orc.OracleSim(N0=300, seed=21, rng_mode=1, Om=3.0, OmDP=2.0)
    for x in (s, o2):
        x.set_state(st["R"], st["V"], psi, st["tPart"] + 0.01, 0.3)
        x.set_forces(st["F"])
        x.qstep_index = 1000
    njump = 0
    for _ in range(40):
        s.qstep(); o2.qstep()
    a, b = s.get_state(), o2.get_state()
    njump = int((b["tPart"] < 0.002).sum())
    assert njump > 5                                   # the branch really ran
    assert np.array_equal(a["tPart"] < 0.002, b["tPart"] < 0.002)
    assert np.abs(a["psi"] - b["psi"]).max() < 1e-10
    assert np.abs(a["V"] - b["V"]).max() < 1e-12


@pytest.mark.parametrize("qt,qt_math", [(1, 0), (1, 1), (1, 2), (0, 0), (0, 2)])
def test_md_steps_short_horizon(eng, orc, qt, qt_math):
    kw = dict(N0=500, seed=77, rng_mode=1, qt_enabled=qt)
    s = eng.Simulation(**kw).init()
    s.set_option("qt_math", qt_math)
    o = orc.OracleSim(nthreads=8, **kw).init()
    s.md_steps(3); o.md_steps(3)
    a, b = s.get_state(), o.get_state()
    assert a["t"] == b["t"]
    assert np.abs(a["R"] - b["R"]).max() < 1e-10
    assert np.abs(a["V"] - b["V"]).max() < 1e-10
    if qt:
        assert np.abs(a["psi"] - b["psi"]).max() < 1e-9
        assert np.array_equal(a["tPart"] == 0, b["tPart"] == 0)


QTK_LANES_IM_EDZ = 1         # mdqt_internal.hpp QTKernel: k_substeps_lanes_im<true, true, true> (no renorm)
QTK_LANES_IM_EDZ_RN = 7      # the same instance with reNormalizewvFns on


def test_c2_headline_qt_instance_matches_oracle(eng, orc):
    """BASELINE configs[1] (C2) exactly as bench.py runs it — N0 = 3500, seed 12346, job 1,
    Philox (rng_mode 1), every option at its default — against the oracle over 3 MD steps with
    quantum jumps.  The production launch must be the one the headline number times:
    k_substeps_lanes_im<true, true, true> (FAST + IM01 + EDZ, no renormalisation: the reference's
    reNormalizewvFns = false) summing all 56 Newton-3 tile slots in its
    lane-distributed prologue (lane k: slots k, k + 16, k + 32, k + 48 — all 16 lanes busy only
    at >= 49 slots) — 57 with the split tile pairs' extra slot (force_tile_split, on 256 CUs) — so
    a slot-sum bug shared with the thread-per-ion kernel cannot hide behind a self-comparison.
    SpeedUp:438-717 (qstep), :1369-1377 (the MD step's cadence)."""
    kw = dict(N0=3500, seed=12346, job=1, rng_mode=1)
    s = eng.Simulation(**kw).init()
    o = orc.OracleSim(nthreads=8, **kw).init()
    assert s.N == o.N == 3573
    s.md_steps(1); o.md_steps(1)            # t = 0 interval: the general instance (non-moving drift)
    assert s.const("qt_kernel") != QTK_LANES_IM_EDZ
    s.md_steps(2); o.md_steps(2)
    assert s.const("force_scheme") == 2 and s.const("force_slots") == 56
    assert s.const("qt_kernel") == QTK_LANES_IM_EDZ, s.const("qt_kernel")
    assert s.const("qt_kernel_nseg") == 56 + (s.const("force_tile_split_pairs") > 0)   # + the split's slot
    a, b = s.get_state(), o.get_state()
    assert a["t"] == b["t"] and s.qstep_index == o.qstep_index == 75
    jumped_a = a["tPart"] < 3 * 25 * 8e-5 - 1e-12
    jumped_b = b["tPart"] < 3 * 25 * 8e-5 - 1e-12
    assert jumped_b.sum() > 50                       # the jump branch ran in every launch
    assert np.array_equal(jumped_a, jumped_b)
    assert np.array_equal(a["tPart"] == 0, b["tPart"] == 0)
    dR, dV = np.abs(a["R"] - b["R"]).max(), np.abs(a["V"] - b["V"]).max()
    dpsi = np.abs(a["psi"] - b["psi"]).max()
    dF = rel(a["F"], b["F"])
    print(f"C2 headline instance: N={s.N} jumps={int(jumped_b.sum())} |dR|={dR:.2e} |dV|={dV:.2e} "
          f"|dpsi|={dpsi:.2e} F rel={dF:.2e}")
    assert dR <= 1e-10 and dV <= 1e-10
    assert dpsi <= 1e-9
    assert dF <= 1e-12
    s.close()


@pytest.mark.parametrize("N0", [30, 45])
def test_newton3_tiles_single_slot(eng, N0):
    """force_scheme 2 with one tile (N <= 64): the kernel writes F itself (no pending slot), so
    every substep instance — including the production FAST launch, which takes nseg == 1 as
    'F already summed' — integrates with this step's forces: equal to the rows scheme (one
    segment: ascending j) up to summation order"""
    out = []
    for scheme in (1, 2):
        s = eng.Simulation(N0=N0, seed=3).init()
        s.set_option("force_scheme", scheme)
        assert s.const("force_scheme") == scheme
        if scheme == 2:
            assert s.N <= 64 and s.const("force_slots") == 1
        s.md_steps(4)
        s.synchronize()
        if scheme == 2:
            assert s.const("qt_kernel") == QTK_LANES_IM_EDZ
        out.append(s.get_state())
        s.close()
    a, b = out
    assert rel(a["F"], b["F"]) < 1e-13
    assert np.abs(a["V"] - b["V"]).max() < 1e-11
    assert np.abs(a["R"] - b["R"]).max() < 1e-11


PUMP = [(1, dict(Om=0.7, detuning=-2.5)), (2, dict(Om=2.0, detuning=0.0)), (3, dict(Om=1.3, detuning=-1.0))]


@pytest.mark.parametrize("model,kw", PUMP)
def test_pump_qstep_matches_oracle(eng, orc, model, kw):
    """optical-pumping qstep (randomFrozenStartTag408Linear/408Quad/422Linear.cpp) vs the oracle"""
    kw = dict(kw, qt_model=model, N0=300, seed=21, rng_mode=1)
    o = orc.OracleSim(nthreads=4, **kw).init()
    o.md_steps(3)
    st = o.get_state()
    s = eng.Simulation(**kw)
    s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    s.set_forces(st["F"])
    s.qstep_index = o.qstep_index
    for _ in range(5):
        s.qstep(); o.qstep()
    a, b = s.get_state(), o.get_state()
    assert np.abs(a["psi"] - b["psi"]).max() < 1e-12
    assert np.array_equal(a["V"], b["V"])            # no optical force, no jump kick
    assert np.array_equal(a["tPart"] == 0, b["tPart"] == 0)
    n = 5 if model == 3 else 7
    assert np.all(a["psi"][:, n:, :] == 0)


@pytest.mark.parametrize("model,kw", PUMP)
def test_pump_jumps_and_md_steps(eng, orc, model, kw):
    """forced P population: many jumps through the model's jump table; then 3 MD steps"""
    kw = dict(kw, qt_model=model, N0=400, seed=5, rng_mode=1)
    o = orc.OracleSim(nthreads=4, **kw).init()
    st = o.get_state()
    n = 5 if model == 3 else 7
    rng = np.random.default_rng(model)
    z = np.zeros((st["psi"].shape[0], 12), complex)
    z[:, :n] = rng.normal(size=(z.shape[0], n)) + 1j * rng.normal(size=(z.shape[0], n))
    z /= np.linalg.norm(z, axis=1, keepdims=True)
    psi = np.stack([z.real, z.imag], -1)
    s = eng.Simulation(**kw)
    for x in (s, o):
        x.set_state(st["R"], st["V"], psi, st["tPart"], 0.0)
    s.md_steps(3); o.md_steps(3)
    a, b = s.get_state(), o.get_state()
    njump = int((b["tPart"] < 3 * 25 * 8e-5 - 1e-12).sum())
    assert njump > 20
    assert np.array_equal(a["tPart"] < 3 * 25 * 8e-5 - 1e-12, b["tPart"] < 3 * 25 * 8e-5 - 1e-12)
    assert np.abs(a["psi"] - b["psi"]).max() < 1e-9
    assert np.abs(a["R"] - b["R"]).max() < 1e-10
    assert np.abs(a["V"] - b["V"]).max() < 1e-10


@pytest.mark.parametrize("model,kw", PUMP)
def test_pump_lane_and_thread_kernels_bit_identical(eng, model, kw):
    sims = []
    for mode in (1, 2):
        s = eng.Simulation(N0=500, seed=31, qt_model=model, **kw).init()
        s.set_option("substep_kernel", mode)
        s.md_steps(3)
        sims.append(s.get_state())
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(sims[0][k], sims[1][k]), k


@pytest.mark.parametrize("model,kw", PUMP)
def test_tag_spin_up_matches_oracle(eng, orc, model, kw):
    """measureSpinUps / tagParticles: same state, same draws -> the same tags"""
    kw = dict(kw, qt_model=model, N0=2000, seed=44, rng_mode=1)
    o = orc.OracleSim(nthreads=4, **kw).init()
    o.md_steps(2)
    st = o.get_state()
    s = eng.Simulation(**kw)
    s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    s.qstep_index = o.qstep_index
    ta, na = s.tag_spin_up()
    tb, nb = o.tag_spin_up()
    assert na == nb and np.array_equal(ta, tb)
    assert 0 < na < len(ta)


def test_pump_models_reject_unsupported_modes(eng):
    s = eng.Simulation(N0=200, qt_model=1)
    with pytest.raises(RuntimeError):
        s.set_option("qt_math", 0)
    with pytest.raises(RuntimeError):
        eng.Simulation(N0=200, qt_model=1, rng_mode=0)
    with pytest.raises(RuntimeError):
        eng.Simulation(N0=200).tag_spin_up()


def test_substeps_fusion_equals_single_substeps(eng):
    """one fused launch of n substeps == n launches of one (bit for bit)"""
    a = eng.Simulation(N0=400, seed=5).init()
    b = eng.Simulation(N0=400, seed=5).init()
    a.forces(); b.forces()
    a.substeps(25)
    for _ in range(25):
        b.substeps(1)
    sa, sb = a.get_state(), b.get_state()
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(sa[k], sb[k]), k
    c = eng.Simulation(N0=400, seed=5).init()
    c.forces()
    for _ in range(25):
        c.step(); c.qstep()
    sc = c.get_state()
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(sa[k], sc[k]), k


@pytest.mark.parametrize("N0,extra", [(500, {}), (3500, {}), (300, dict(Om=3.0, OmDP=2.0, reNormalizewvFns=1)),
                                      (300, dict(fracOfSig=0.4, detuningDP=-0.5))])
@pytest.mark.parametrize("qt_math", [0, 1, 2])
def test_lane_and_thread_qt_kernels_bit_identical(eng, N0, extra, qt_math):
    """k_substeps_lanes (16 lanes per ion) performs exactly k_substeps' operations"""
    sims = []
    for mode in (1, 2):
        s = eng.Simulation(N0=N0, seed=31, **extra).init()
        s.set_option("substep_kernel", mode)
        s.set_option("qt_math", qt_math)
        s.md_steps(3)
        if mode == 2 and qt_math == 2 and extra.get("reNormalizewvFns"):
            assert s.const("qt_kernel") == QTK_LANES_IM_EDZ_RN     # not the production (no-renorm) code
        sims.append(s.get_state())
    a, b = sims
    jumped = (a["tPart"] < 3 * 0.002).sum()
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(a[k], b[k]), (k, jumped)


def test_lane_kernel_large_phase_fallback_bit_identical(eng):
    """coupling phases (SpeedUp:508) beyond the table reduction's 2^20 (an ion long without a
    jump): the production lane instance's wave-uniform phase bound must send those waves through
    the loop with the library fallback — bit-identical to the thread kernel, which checks every
    substep; the waves whose bound holds run the loop without it"""
    sims = []
    for mode in (1, 2):
        s = eng.Simulation(N0=3500, seed=31).init()
        s.md_steps(2)
        st = s.get_state()
        tp = st["tPart"].copy()
        tp[::97] += 3.0e6                          # a few ions per few waves: |phi| far above 2^20
        s.set_state(st["R"], st["V"], st["psi"], tp, st["t"])
        s.set_option("substep_kernel", mode)
        s.md_steps(2)
        if mode == 2:
            assert s.const("qt_kernel") == QTK_LANES_IM_EDZ
        sims.append((s.get_state(), tp, s.const("plasVelToQuantVel"), s.const("gamToEinsteinFreq")))
    (a, tp, pv2q, g), (b, _, _, _) = sims
    cphi = 2. * (1. + 0.395) * g                    # FastTab::cphi (kRat 0.395, SpeedUp:146)
    phi = np.abs(a["V"][0] * pv2q * cphi * tp)
    assert (phi > 2. ** 21).sum() >= 10            # the fallback ran for these ions
    for k in ("R", "V", "psi", "tPart"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("N0,extra,qt_math", [(300, {}, 0), (500, dict(Om=3.0, OmDP=2.0), 0), (3500, {}, 0),
                                              (500, dict(Om=3.0, OmDP=2.0), 2)])
def test_drand48_reference_order_matches_oracle(eng, orc, N0, extra, qt_math):
    """rng_mode 0: the reference's own drand48 stream consumed in its order (1 draw per ion,
    4-5 per quantum jump) — same jumps, same stream position, same trajectory as the oracle's
    reference-order restatement"""
    kw = dict(N0=N0, seed=12346, rng_mode=0, **extra)
    s = eng.Simulation(**kw).init()
    s.set_option("qt_math", qt_math)            # 0: the reference's exact operations
    o = orc.OracleSim(**kw).init()
    assert s.drand48_state == orc.lib().orc_get_drand48_state(o.h)
    s.md_steps(4); o.md_steps(4)
    a, b = s.get_state(), o.get_state()
    assert s.drand48_state == orc.lib().orc_get_drand48_state(o.h)    # same number of draws
    assert np.array_equal(a["tPart"] == 0, b["tPart"] == 0) or np.array_equal(a["tPart"] < 1e-3, b["tPart"] < 1e-3)
    assert np.abs(a["psi"] - b["psi"]).max() < 1e-9
    assert np.abs(a["V"] - b["V"]).max() < 1e-10
    assert np.abs(a["R"] - b["R"]).max() < 1e-10


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_local_group_bit_identical(eng, world):
    """the sharded data path (slab layout [world][3][S], all-gather of positions, owner-computes
    force rows, global-id RNG) run as an in-process rank group is bit-identical to world 1"""
    from mdqtplasmasims_amd.engine import comm_init_local
    kw = dict(N0=700, seed=9)
    ref = eng.Simulation(**kw).init()
    ref.set_option("force_scheme", 1)          # the owner-computes rows every shard runs
    ref.md_steps(3)
    rs = ref.get_state()
    st = eng.Simulation(**kw).init().get_state()
    sims = [eng.Simulation(world_size=world, rank=r, **kw) for r in range(world)]
    for s in sims:
        s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    comm_init_local(sims)
    for _ in range(3):
        for s in sims:
            s.allgather_positions()
        for s in sims:
            s.forces()
        for s in sims:
            s.substeps(25)
    for s in sims:
        lo, hi = s.slab_bounds()
        a = s.get_state()
        assert hi > lo
        for k in ("R", "V"):
            assert np.array_equal(a[k][:, lo:hi], rs[k][:, lo:hi]), k
        for k in ("psi", "tPart"):
            assert np.array_equal(a[k][lo:hi], rs[k][lo:hi]), k
        assert a["t"] == rs["t"]


# ---------------------------------------------------------------------------------------------
# observables and files
# ---------------------------------------------------------------------------------------------

def test_observables_match_oracle(eng, orc):
    kw = dict(N0=500, seed=8, rng_mode=1)
    s = eng.Simulation(**kw).init()
    o = orc.OracleSim(nthreads=8, **kw).init()
    s.md_steps(2); o.md_steps(2)
    st = o.get_state()
    s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])   # identical state
    a7, aP, ap = s.observables()
    b7, bP, bp = o.observables()
    assert a7[0] == b7[0]
    idx = [1, 2, 3, 4, 6]                          # EkinX, EkinY, EkinZ, Epot, <vx>
    assert np.allclose(a7[idx], b7[idx], rtol=1e-12, atol=1e-15)
    # Etot - Epot0 cancels to ~1e-7 of Epot: compare on the scale of the terms
    assert abs(a7[5] - b7[5]) <= 1e-12 * abs(b7[4])
    assert rel(aP, bP) < 1e-12
    assert np.allclose(ap, bp, rtol=1e-14, atol=1e-16)
    assert abs(s.Epotential() - o.epotential()) <= 1e-12 * abs(o.epotential())


def test_kde_skipping_matches_dense_sum(eng, orc):
    """output()'s Gaussian KDE (SpeedUp:958-979) on the device skips, per wave, ions whose terms are
    exact zeros on all its bins (|b -+ v| >= kKdeSkip = 0.0773, beyond exp's underflow for
    V2 = 1/(2 0.002^2); mdqt_internal.hpp asserts the threshold against V2): against the oracle's
    dense sum on velocities spread over and beyond the 2001 bins, with ions placed just inside and
    just outside the skip distance of bin centres"""
    kw = dict(N0=500, seed=8, rng_mode=1)
    o = orc.OracleSim(nthreads=8, **kw).init()
    st = o.get_state()
    rng = np.random.default_rng(2)
    V = rng.uniform(-5.3, 5.3, st["V"].shape)
    n = V.shape[1] // 4
    bins = rng.integers(0, 2001, (3, n)) * 0.0025
    V[:, :n] = bins + rng.choice([-1.0, 1.0], (3, n)) * (0.0773 + rng.choice([-1e-4, 1e-4, 0.0], (3, n)))
    s = eng.Simulation(**kw)
    for x in (s, o):
        x.set_state(st["R"], V, st["psi"], st["tPart"], st["t"])
    _, aP, _ = s.observables(pops=False)
    _, bP, _ = o.observables(pops=False)
    assert rel(aP, bP) < 1e-12
    s.close()


@pytest.mark.parametrize("N0", [500, 3500])
def test_epotential_newton3_tiles_match_rows(eng, N0):
    """Epotential() on the Newton-3 tiles (each distinct pair once, world 1 default) against the
    owner-computes rows (every ordered pair): the same sum up to summation order"""
    s = eng.Simulation(N0=N0, seed=29).init()
    s.md_steps(2)
    assert s.const("force_scheme") == 2 and s.const("potential_n3") == 1
    e3 = s.Epotential()
    s.set_option("potential_n3", 0)
    er = s.Epotential()
    s.close()
    assert abs(e3 - er) <= 1e-14 * abs(er), (e3, er)


def _read_dir(d):
    out = {}
    for f in sorted(os.listdir(d)):
        out[f] = open(os.path.join(d, f)).read()
    return out


def test_run_writes_reference_layout(eng, orc, tmp_path):
    kw = dict(N0=60, tmax=0.09, sampleFreq=5, seed=99, job=3, rng_mode=1)
    s = eng.Simulation(saveDirectory=str(tmp_path / "gpu") + "/", **kw)
    s.run()
    o = orc.OracleSim(saveDirectory=str(tmp_path / "cpu") + "/", **kw)
    assert o.run() == 0
    A, B = _read_dir(s.save_directory), _read_dir(o.save_directory)
    assert s.save_directory.endswith(
        "Ge10Density2000E+11Sig040Te19SigFrac0DetSP-100DetDP100OmSP100OmDP100NumIons60/job3/")
    assert sorted(A) == sorted(B)
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
        # %lg keeps 6 significant digits: files agree to the printed precision
        assert np.allclose(xa, xb, rtol=2e-5, atol=1e-9 * max(1.0, np.abs(xb).max())), f


def test_init_parallel_sampling_matches_sequential(eng):
    """init()'s drand48 rejection sampling in parallel (option init_threads, default auto) equals
    the sequential walk (init_threads 1) bit for bit, incl. the stream state qsteps continue from"""
    out = []
    for th in (1, 6):
        s = eng.Simulation(N0=3500, seed=12346, rng_mode=0)
        s.set_option("init_threads", th)
        s.init()
        st = s.get_state()
        out.append((s.N, st["R"], st["psi"], s.drand48_state))
        s.close()
    (n1, R1, p1, x1), (n2, R2, p2, x2) = out
    assert n1 == n2 == 3573
    assert np.array_equal(R1, R2) and np.array_equal(p1, p2) and x1 == x2


def test_run_files_are_lg_of_the_final_state(eng, tmp_path):
    """mdqt_run's files come from the background writers (mdqt_writer.hpp): byte for byte the
    "%lg" text of the state the run ends with (SpeedUp:747, :777-779)."""
    kw = dict(N0=300, tmax=0.1, sampleFreq=10, seed=21, job=2, rng_mode=1)
    s = eng.Simulation(saveDirectory=str(tmp_path) + "/", **kw)
    s.run()
    s.flush_files()
    st = s.get_state()
    c0 = s.counters()["c0"]
    R, V, psi = st["R"], st["V"], st["psi"]
    N = s.N
    d = s.save_directory
    want = "".join("".join("%g\t" % R[k, i] for k in range(3)) + "".join("%g\t" % V[k, i] for k in range(3)) + "\n"
                   for i in range(N))
    assert open(os.path.join(d, "conditions_timestep%06d.dat" % c0)).read() == want
    P = psi.reshape(N, -1)
    want = "".join("".join("%g\t" % v for v in P[i]) + "\n" for i in range(N))
    assert open(os.path.join(d, "wvFns_timestep%06d.dat" % c0)).read() == want
    assert open(os.path.join(d, "ions_timestep%06d.dat" % c0)).read() == "%d\t%d" % (N, s.counters()["counter"])
    # one velocity distribution per output, each 2001 rows
    for n in range(s.counters()["counter"]):
        assert len(open(os.path.join(d, "vel_distZ_time%06d.dat" % n)).read().splitlines()) == 2001


def test_resume_roundtrip(eng, tmp_path):
    kw = dict(N0=60, tmax=0.05, sampleFreq=1000, seed=5, job=1, saveDirectory=str(tmp_path) + "/")
    s = eng.Simulation(**kw)
    s.run()
    c0 = s.counters()["c0"]
    st = s.get_state()
    r = eng.Simulation(newRun=0, c0=c0, **{k: v for k, v in kw.items()})
    r.setup_directories()
    r.readConditions(c0)
    st2 = r.get_state()
    assert r.N == s.N
    assert np.allclose(st2["R"], st["R"], rtol=1e-5, atol=1e-6)
    assert np.allclose(st2["psi"], st["psi"], rtol=1e-5, atol=1e-6)
    assert r.t == (c0 - 9.0) * 0.002 + 0.02          # SpeedUp:789
    assert (st2["tPart"] == 0).all()


def test_cli_runs(eng, tmp_path):
    import subprocess
    from mdqtplasmasims_amd import CLI_PATH
    r = subprocess.run([CLI_PATH, "2", "--N0=80", "--tmax=0.02", "--seed=4",
                        f"--saveDirectory={tmp_path}/"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = tmp_path / "Ge10Density2000E+11Sig040Te19SigFrac0DetSP-100DetDP100OmSP100OmDP100NumIons80" / "job2"
    assert (d / "ions_timestep000010.dat").exists()


# ---------------------------------------------------------------------------------------------
# size-independent properties at the benchmark sizes
# ---------------------------------------------------------------------------------------------

def test_momentum_conservation_of_forces_c2(eng):
    s = eng.Simulation(N0=3500, seed=12346).init()
    s.forces()
    F = s.get_state()["F"]
    assert np.abs(F.sum(axis=1)).max() < 1e-10 * np.abs(F).sum() / F.shape[1]


def test_norm_decay_and_partition_of_qt(eng):
    """the no-jump propagator keeps |psi| ~ 1 (normalised non-Hermitian step, App. A) and
    populations stay in [0,1] over an MD step at the C2 size"""
    s = eng.Simulation(N0=3500, seed=12346).init()
    s.md_steps(2)
    st = s.get_state()
    nrm = (st["psi"] ** 2).sum(axis=(1, 2))
    assert np.abs(nrm - 1).max() < 1e-3
    o7, P, pops = s.observables()
    assert np.all(pops >= -1e-15) and np.all(pops.sum(1) < 1.001)


@pytest.mark.parametrize("N0", [500, 3500])
def test_fused_md_step_bit_identical(eng, N0):
    """one MD step as ONE launch (k_md_step: the tile pairs, then the QT workgroups waiting on the
    per-tile arrival counts; option fused_step, default off) against forces() + substeps(ratio) as
    two launches: bit for bit over MD steps with quantum jumps (the first step, t = 0, is never
    fused — the non-moving drift branch)"""
    out = []
    for fu in (0, 1):
        s = eng.Simulation(N0=N0, seed=73).init()
        s.set_option("force_tile_split", 0)            # (the fused launch takes the plain tile-pair table)
        s.set_option("fused_step", fu)
        assert s.const("fused_step") == fu
        s.md_steps(30)
        s.synchronize()
        assert s.const("md_step_fused") == fu
        out.append(s.get_state())
        s.close()
    a, b = out
    for k in ("R", "V", "F", "psi", "tPart"):
        assert np.array_equal(a[k], b[k]), k
    assert (a["tPart"] < 30 * 0.002 - 1e-9).sum() > 0          # jumps happened


def test_lane_kernel_im01_instance_matches_general(eng):
    """the FAST lane instance without the real-part FMAs of the purely imaginary static coupling
    slots (QTConst::im01, the production model-0 launch) against the general FAST instance: the
    dropped terms are +-0 * y, so the trajectories agree bit for bit (up to the sign of zero)
    over MD steps with quantum jumps"""
    out = []
    for im in (1, 0):
        s = eng.Simulation(N0=700, seed=91).init()
        assert s.const("qt_im01") == 1                 # model 0: -i h H with real couplings
        s.set_option("qt_im01", im)
        assert s.const("qt_im01") == im
        s.md_steps(30)
        s.synchronize()
        out.append(s.get_state())
        s.close()
    a, b = out
    for k in ("R", "V", "F", "psi", "tPart"):
        assert np.array_equal(a[k], b[k]), k
    assert (a["tPart"] < 30 * 0.002 - 1e-9).sum() > 0          # jumps happened


def test_fused_md_step_run_files_identical(eng, tmp_path):
    """mdqt_run (the reference's main loop) fuses whole intervals between outputs: the files of a
    run are byte-identical with and without the fused launch"""
    kw = dict(N0=300, tmax=0.3, sampleFreq=7, seed=5, job=2, rng_mode=1)
    dirs = []
    for fu in (0, 1):
        s = eng.Simulation(saveDirectory=str(tmp_path / f"f{fu}") + "/", **kw)
        s.set_option("force_tile_split", 0)
        s.set_option("fused_step", fu)
        s.run()
        dirs.append(s.save_directory)
        s.close()
    A, B = _read_dir(dirs[0]), _read_dir(dirs[1])
    assert sorted(A) == sorted(B) and len(A) > 5
    for f in A:
        assert A[f] == B[f], f


@pytest.mark.parametrize("N0", [500, 3500])
def test_overlapped_md_step_bit_identical(eng, N0):
    """mdqt_md_steps with the force and QT launches overlapped (QT prologue on its own stream, a
    device-side arrival count instead of the kernel boundary, write-through partials) is the same
    arithmetic as the sequential order: bit for bit, over MD steps with quantum jumps"""
    out = []
    for ov in (0, 1):
        s = eng.Simulation(N0=N0, seed=71).init()
        s.set_option("force_tile_split", 0)            # (the overlapped steps take the plain tile-pair table)
        s.set_option("overlap", ov)
        s.md_steps(30)
        s.synchronize()
        out.append(s.get_state())
        s.close()
    a, b = out
    for k in ("R", "V", "F", "psi", "tPart"):
        assert np.array_equal(a[k], b[k]), k
    assert (a["tPart"] < 30 * 0.002 - 1e-9).sum() > 0          # jumps happened

def test_tile_split_of_the_last_round(eng):
    """the tile kernel's last round of workgroups: the whole tile pairs left in it run in parts
    (mdqt_engine.cpp tile_split_count; C2 on 256 CUs: 1,596 workgroups, 60 in the last round, 56 of
    them diagonal — 4 split), later parts' rows in extra slots: the same pair terms, summed in another
    order — within rounding of the plain table; halves (option 1) change only the split pairs' tiles,
    quarters (option 2) halve every diagonal tile as well"""
    s = eng.Simulation(N0=3500, seed=12346, job=1).init()     # bench.py's C2: N = 3,573, 56 tiles
    assert s.N == 3573
    out, ks = {}, {}
    for sp in (2, 1, 0):
        s.set_option("force_tile_split", sp)
        ks[sp] = int(s.const("force_tile_split_pairs"))
        s.forces()
        out[sp] = s.get_state()["F"]
    cus = s.const("device_cus")
    s.close()
    if cus == 256:                                    # MI355X
        assert ks[1] == 4 and ks[2] == 4
    assert ks[0] == 0
    scale = np.abs(out[0]).max()
    for sp in (1, 2):
        d = np.abs(out[sp] - out[0])
        print(f"C2 split {sp} ({ks[sp]} tile pairs): max|dF|/max|F| = {d.max() / scale:.3e}")
        assert d.max() <= 1e-13 * scale
        assert ks[sp] == 0 or d.max() > 0              # (the split ran: another summation order)
    assert not np.abs(out[1] - out[0])[:, 2 * ks[1] * 64:].any()   # halves: only the split pairs' tiles


def test_tile_split_fixed_cu_count(eng):
    """force_split_cus: the split table cut for a given CU count on any device — 256
    gives the MI355X table bit for bit whatever the device, another count another table (a 304-CU
    device's: C2's 1,596 workgroups leave 76 in the last round, 20 whole pairs) within rounding"""
    s = eng.Simulation(N0=3500, seed=12346, job=1).init()
    out, ks = {}, {}
    for n in (0, 256, 304):
        s.set_option("force_split_cus", n)
        assert s.const("force_split_cus") == n
        ks[n] = int(s.const("force_tile_split_pairs"))
        s.forces()
        out[n] = s.get_state()["F"]
    cus = s.const("device_cus")
    s.close()
    assert ks[256] == 4
    if cus == 256:
        assert ks[0] == 4 and np.array_equal(out[0], out[256])
    scale = np.abs(out[256]).max()
    assert ks[304] != ks[256]
    assert np.abs(out[304] - out[256]).max() <= 1e-13 * scale
