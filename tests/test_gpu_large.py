"""The HIP path at BASELINE.json's large configurations (C3, C4, C5), checked against
the oracle on sampled ions (the full O(N^2) oracle is hours at N = 1e6).

  C3  N0 = 100,000  MD-only, Ge = 1/12 (kappa = 0.5)      Newton-3 block pairs, one GPU
  C4  N0 = 1,000,000 MD-only, Ge = 1/12                  Newton-3 block pairs, one GPU (~12 GB of slots)
  C5  N0 = 250,000  full MDQT, detuningDP = +1           Newton-3 block pairs + one fused 25-substep launch
  1M  N0 = 1,000,000 full MDQT (C2's laser parameters)   north_star's second size: QT on at N = 1e6

Per config:
  * forces() on the reference's init() state (C5: after 20 MD steps, so that the interval below
    has quantum jumps): GPU F of ~1,000 sampled ions (one per 1,024 ions, the ragged last tile, both sides of the NB/2 half-shell boundary, random others) against
    the oracle's rows over all j (orc_forces_index: the reference's pair terms, compensated sum so
    that the check sees the GPU's rounding, not N eps of the oracle's own);
    gate: max |dF| <= 1e-12 x max |F| over the sample (stated tolerance: the GPU sums N/2 terms per
    ion through ~NB/2 block slots; measured ~1e-14);
  * momentum: |sum_i F_i| <= 1e-9 x mean |F_i| (each distinct pair is evaluated once, +f and -f;
    only the summation rounding of ~N^2/2 terms remains);
  * MD-only (C3, C4): one MD step's 25 drift substeps with F frozen are exact arithmetic (step(),
    SpeedUp:356-430): sampled ions equal the oracle's step() bit for bit;
  * C5: one fused 25-substep launch (step()+qstep(), SpeedUp:356-717) with the GPU's F frozen on the
    sampled ions against the oracle run on those ions alone (ions are independent between force
    calls; the oracle draws the same Philox uniforms keyed by the global ion id):
    tPart (jump pattern) and R, V, psi within the per-qstep gates.
"""
import os

import numpy as np
import pytest

CONFIGS = {
    "C3": dict(N0=100000, Ge=1.0 / 12, qt_enabled=0),
    "C5": dict(N0=250000, detuningDP=1.0, qt_enabled=1),
    "C4": dict(N0=1000000, Ge=1.0 / 12, qt_enabled=0),
    "1M": dict(N0=1000000, qt_enabled=1),
}
SEED = 12346


def threads():
    return max(1, min(16, os.cpu_count() or 1))


BLOCK = 512                                         # ions per block of the block kernel (8 tiles)


def sample_ions(N, nsamp, rng):
    """one ion per 1,024 ions (every other block), the ragged last tile, the blocks around NB/2,
    random others"""
    NB = (N + BLOCK - 1) // BLOCK
    idx = [b * 1024 + int(rng.integers(0, min(1024, N - b * 1024))) for b in range((N + 1023) // 1024)]
    idx += list(range(max(0, N - 64), N))                          # ragged last tile
    for b in (NB // 2 - 1, NB // 2, NB // 2 + 1, NB - 1, 0):       # half-shell boundary blocks
        if 0 <= b < NB:
            lo = b * BLOCK
            idx += list(range(lo, min(N, lo + 8))) + list(range(max(lo, min(N, lo + BLOCK) - 8), min(N, lo + BLOCK)))
    rest = nsamp - len(set(idx))
    if rest > 0:
        idx += list(rng.integers(0, N, rest))
    return np.array(sorted(set(int(i) for i in idx)), dtype=np.int64)


def test_forces_index_matches_full_rows(orc):
    """CPU: the indexed, compensated rows equal the plain rows to rounding (no GPU)"""
    rng = np.random.default_rng(3)
    L = 24.474785
    R = rng.uniform(0, L, (3, 900))
    idx = np.array([0, 1, 63, 64, 450, 899])
    A = orc.forces_index(R, idx, L, 1.8257418583505538, nthreads=2)
    B = orc.forces_raw(R, L, 1.8257418583505538)[:, idx]
    assert np.abs(A - B).max() <= 1e-13 * np.abs(B).max()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C3", "C5", "C4", "1M"])
def test_large_config_forces_and_interval(cfg, orc):
    import mdqtplasmasims_amd as M
    if M.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked tests")
    kw = dict(CONFIGS[cfg])
    qt = kw["qt_enabled"]
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **kw).init()
    if qt:
        s.md_steps(20 if cfg != "1M" else 8)            # P populations build up: quantum jumps occur
    N = s.N
    assert s.const("force_scheme") == 3                 # Newton-3 block pairs above 65,536 ions
    L, lDeb = s.const("L"), s.const("lDeb")
    s.forces()
    st = s.get_state()
    R, F = st["R"], st["F"]
    rng = np.random.default_rng(11)
    idx = sample_ions(N, 1024 if N < 500000 else 640, rng)
    G = orc.forces_index(R, idx, L, lDeb, nthreads=threads())
    dabs = np.abs(F[:, idx] - G).max()
    err = dabs / np.abs(G).max()
    # the error-bounded tail (force_tail_exp, default 12): tile pairs >= r_t apart are skipped, every
    # ion's force moves by at most `bound` (mdqt_engine.cpp tail_radius; 0 where r_t = L/2)
    # and the far pair form (force_far_exp, default 13): <= far bound more
    rt, bound = s.const("force_skip_radius"), s.const("force_tail_bound")
    rf, fbound = s.const("force_far_radius"), s.const("force_far_bound")
    print(f"{cfg}: N={N} NB={(N + BLOCK - 1) // BLOCK} N%64={N % 64} sampled {len(idx)}: max|dF|/max|F| = {err:.3e}, "
          f"max|dF| = {dabs:.3e}; skip radius {rt:.3f} (L/2 {L / 2:.3f}), tail bound {bound:.2e}; "
          f"far radius {rf:.3f}, far bound {fbound:.2e}")
    vbound = s.const("force_vfar_bound") + s.const("force_ufar_bound") + s.const("force_mid_bound")
    assert err <= 1e-12
    assert dabs <= bound + fbound + vbound + 1e-13 * np.abs(G).max()
    mom = np.abs(F.sum(axis=1)).max() / (np.abs(F).sum() / N)
    print(f"{cfg}: |sum F| / mean|F| = {mom:.3e}")
    assert mom <= 1e-9
    # one MD interval (25 substeps) with F frozen, sampled ions vs the oracle on those ions alone
    ratio = int(s.const("plasmaToQuantumTimestepRatio"))
    q0 = s.qstep_index
    s.substeps(ratio)
    after = s.get_state()
    o = orc.OracleSim(seed=SEED, job=1, rng_mode=1, nthreads=threads(), **kw)
    assert o.const("L") == L
    n = len(idx)
    o.set_state(R[:, idx], st["V"][:, idx], st["psi"][idx], st["tPart"][idx], st["t"])
    o.set_forces(F[:, idx])
    o.set_ion_ids(idx)
    o.qstep_index = q0
    o.substeps(ratio)
    b = o.get_state()
    assert b["t"] == after["t"]
    if not qt:
        assert np.array_equal(after["R"][:, idx], b["R"]) and np.array_equal(after["V"][:, idx], b["V"])
    else:
        assert np.abs(after["tPart"][idx] - b["tPart"]).max() <= 1e-15        # same jump substeps
        dR = np.abs(after["R"][:, idx] - b["R"]).max()
        dV = np.abs(after["V"][:, idx] - b["V"]).max()
        dpsi = np.abs(after["psi"][idx] - b["psi"]).max()
        print(f"{cfg}: interval of {ratio} substeps on {n} ions: max|dR| {dR:.2e} |dV| {dV:.2e} |dpsi| {dpsi:.2e}, "
              f"ions that jumped {int((b['tPart'] < 0.999 * ratio * s.const('quantumTimestep')).sum())}")
        assert dR <= 1e-12 and dV <= 1e-13 and dpsi <= 1e-11
        assert (b["tPart"] < 0.999 * ratio * s.const("quantumTimestep")).sum() >= 3   # the jump branch ran
    o.close()
    s.close()


@pytest.mark.gpu
def test_force_census_covers_every_pair():
    """mdqt_force_census (the bench's per-tier pair counts): every distinct ion pair of the system is
    in exactly one tile pair of one class — the classes' ion pairs sum to N(N-1)/2 — at C3 (no tail
    skipping: r_t = L/2) and in a world-2 group (the ranks' censuses add up)"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS["C3"]).init()
    N = s.N
    c = s.force_census()
    pairs = sum(v[1] for v in c.values())
    work = sum(v[0] for k, v in c.items() if not k.startswith("skip"))
    print(f"C3 census: " + ", ".join(f"{k} {v[1] / (N * (N - 1) / 2):.3f}" for k, v in c.items())
          + f"; evaluated lane-steps / (N(N-1)/2) = {work / (N * (N - 1) / 2):.3f}")
    assert pairs == N * (N - 1) // 2
    assert c["skip_tail"] == (0, 0) and c["skip_cut"][1] > 0 and c["ufar32_uniform"] == (0, 0)
    st = s.get_state()
    s.close()
    tot = 0
    for r in range(2):
        x = M.Simulation(seed=SEED, job=1, rng_mode=1, world_size=2, rank=r, **CONFIGS["C3"])
        x.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
        tot += sum(v[1] for v in x.force_census().values())
        x.close()
    assert tot == N * (N - 1) // 2


@pytest.mark.gpu
def test_spatial_order_tile_skipping_is_exact(orc):
    """Newton-3 blocks in Hilbert order (mdqt_sort.hip): skipping tile pairs whose boxes are >= L/2
    apart changes nothing (they add exact zeros) — bit for bit against the same order without
    skipping; against the unsorted order the forces agree to rounding (1e-13 of max |F|)"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS["C3"]).init()
    out = {}
    for mode in (1, 2, 0):
        s.set_option("force_sort", mode)
        assert s.const("force_sort") == mode
        s.forces()
        out[mode] = s.get_state()["F"]
    assert np.array_equal(out[1], out[2])
    err = np.abs(out[1] - out[0]).max() / np.abs(out[0]).max()
    print(f"C3 sorted vs unsorted: max|dF|/max|F| = {err:.3e}")
    assert err <= 1e-13
    s.close()


@pytest.mark.gpu
def test_one_axis_image_instance_matches_per_pair_image():
    """force_ax1 (mdqt_forces.hip n3b_pack_class, launch_forces_n3b): a tile pair whose minimum image
    varies on one axis only takes the image per pair on that axis alone and the other two axes'
    multiples once per tile pair, as a uniform-image tile pair does — the same pair terms (SpeedUp:
    218-224), the shifted axes rounded as in the uniform-image tile pairs.  At C3 (skip radius L/2,
    so the instance runs) against force_ax1 0 (every per-pair image on all three axes): within
    rounding, 1e-13 of max |F|"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS["C3"]).init()
    assert s.const("force_ax1") == 1 and s.const("force_skip_radius") == s.const("L") / 2
    out = {}
    for mode in (1, 0):
        s.set_option("force_ax1", mode)
        s.forces()
        out[mode] = s.get_state()["F"]
    err = np.abs(out[1] - out[0]).max() / np.abs(out[0]).max()
    print(f"C3 one-axis image vs per-pair image on all axes: max|dF|/max|F| = {err:.3e}")
    assert err <= 1e-13
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C4", "C5"])
def test_error_bounded_tail_and_far_form(cfg):
    """The error-bounded parts of the Newton-3 block forces against the exact sum to L/2 on EVERY
    ion: the skip radius r_t < L/2 (force_tail_exp 12: |dF_i| <= (N - 1) g(r_t) <= 1e-12,
    mdqt_engine.cpp tail_radius; active at N ~ 1e6), the far pair form beyond r_far (force_far_exp
    13: (N - 1) g(r_far) kFarRelErr <= 1e-13) and the very-far form beyond r_vfar (force_vfar_exp
    13: (N - 1) g(r) ((r/lDeb + 3) kRsqRawErr + kExp5RelErr) <= 1e-13), the ultra-far forms and the
    mid form beyond r_mid (force_mid_exp 13, round 4: (N - 1) g(r) ((r/lDeb + 3)(kRsq1RelErr + 2^-52)
    + kTab4RelErr) <= 1e-13) — each alone and all together, plus the summation-order rounding; r_t
    is a no-op at C3 and C5.  (force_form_mode 0: the a-priori tier radii; mode 1, the default, below)"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS[cfg]).init()
    s.set_option("force_form_mode", 0)                 # (the a-priori tier radii; form mode 1: the test below)
    L = s.const("L")
    rt, tb = s.const("force_skip_radius"), s.const("force_tail_bound")
    rm, mb0 = s.const("force_mid_radius"), s.const("force_mid_bound")
    rf, fb = s.const("force_far_radius"), s.const("force_far_bound")
    rv, vb = s.const("force_vfar_radius"), s.const("force_vfar_bound")
    ru, ub = s.const("force_ufar_radius"), s.const("force_ufar_bound")
    ru32 = s.const("force_ufar32_radius")             # the f32 ultra-far shell (its bound is in ub)
    assert 0 < fb <= 1e-13 and rf < L / 2 and 0 < vb <= 1e-13 and rf < rv < L / 2
    assert 0 < mb0 <= 1e-13 and rm < rf
    assert 0 < ub <= 2e-13 and rf < ru < L / 2 and ru <= ru32 <= L / 2   # ub: f64 + f32 shells, 1e-13 each
    # (C4: the measured bound needs a force call — read after the calls below)
    assert (rt < L / 2) if cfg == "C4" else (tb == 0 and rt == L / 2)
    out = {}
    for te, me, fe, ve, ue in ((12, 13, 13, 13, 13), (0, 0, 13, 0, 0), (0, 0, 0, 13, 0), (0, 0, 0, 0, 13),
                               (12, 0, 0, 0, 0), (0, 13, 0, 0, 0), (0, 0, 0, 0, 0)):
        s.set_option("force_tail_exp", te)
        s.set_option("force_mid_exp", me)
        s.set_option("force_far_exp", fe)
        s.set_option("force_vfar_exp", ve)
        s.set_option("force_ufar_exp", ue)
        s.forces()
        out[te, me, fe, ve, ue] = s.get_state()["F"]
    assert s.const("force_skip_radius") == L / 2 and s.const("force_far_bound") == 0
    assert s.const("force_mid_bound") == 0 and s.const("force_mid_radius") == L / 2
    assert s.const("force_vfar_bound") == 0 and s.const("force_ufar_bound") == 0
    if cfg == "C4":
        # force_tail_mode 1: the bound is what the calls measured — per tile, n_J g(box distance)
        # summed over its skipped tile pairs — kept as a running maximum over the calls (reset by
        # the option change: NaN until a call has measured)
        s.set_option("force_tail_exp", 12)
        assert s.const("force_tail_mode") == 1 and s.const("force_skip_radius") == rt
        assert np.isnan(s.const("force_tail_bound"))
        s.forces()
        tb = s.const("force_tail_bound")
        mb = s.const("force_tail_model_bound")
        print(f"{cfg}: measured tail bound {tb:.3e} (the model chose r_t for {mb:.3e}; a priori (N - 1) g(r_t) "
              f"{(s.N - 1) * (1 / rt + 1 / s.const('lDeb')) * np.exp(-rt / s.const('lDeb')) / rt:.3e}); "
              f"tiles over 1e-12 {s.const('force_tail_fixed_tiles'):.0f}")
        assert 0 < tb <= 1e-12 and 0 < mb <= 1e-12 / 1.25 * (1 + 1e-9)     # kTailMargin
        assert s.const("force_tail_fixed_tiles") == 0 and s.const("force_tail_raw_bound") <= 1e-12
    Fe = out[0, 0, 0, 0, 0]
    scale = 1e-13 * np.abs(Fe).max()
    d = {k: np.abs(v - Fe).max() for k, v in out.items()}
    print(f"{cfg} N={s.N}: r_t {rt:.3f} (bound {tb:.2e}), r_mid {rm:.3f} ({mb0:.2e}), r_far {rf:.3f} ({fb:.2e}), "
          f"r_vfar {rv:.3f} ({vb:.2e}), r_ufar {ru:.3f} ({ub:.2e}), r_ufar32 {ru32:.3f}, L/2 {L / 2:.3f}; max_i |dF_i|: "
          f"all {d[12, 13, 13, 13, 13]:.3e}, mid only {d[0, 13, 0, 0, 0]:.3e}, far only {d[0, 0, 13, 0, 0]:.3e}, "
          f"very far only {d[0, 0, 0, 13, 0]:.3e}, ultra far only {d[0, 0, 0, 0, 13]:.3e}, tail only "
          f"{d[12, 0, 0, 0, 0]:.3e}; max|F| {np.abs(Fe).max():.3e}")
    assert d[12, 13, 13, 13, 13] <= tb + mb0 + fb + vb + ub + scale
    assert d[0, 13, 0, 0, 0] <= mb0 + scale
    assert d[0, 0, 13, 0, 0] <= fb + scale
    assert d[0, 0, 0, 13, 0] <= vb + scale
    assert d[0, 0, 0, 0, 13] <= ub + scale
    assert d[12, 0, 0, 0, 0] <= tb + scale
    s.close()
    if cfg == "C5":                                    # r_t >= L/2 at C3 too: exact skipping only
        x = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS["C3"])
        x.set_state(*_tiny_state(x))
        x.set_option("force_form_mode", 0)               # (the tail's own bound: no measured form sums)
        assert x.const("force_tail_bound") == 0 and x.const("force_skip_radius") == x.const("L") / 2
        x.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C4", "C5"])
def test_form_bound_measured_and_enforced(cfg):
    """force_form_mode 1 and 2 (round 6; 2 the default): the tiers' radii from the density model of the sums the
    plan measures (mdqt_engine.cpp tier_radius) — below the a-priori radii of mode 0 — and every
    sub-block evaluated in an error-bounded form adding n_b g(gap) err_form(gap) to its sub-tiles' sums
    (k_n3b_plan), which k_tail_max holds to force_error_eps (the tail's eps where r_t < L/2 + 10^-13 per
    active tier; mode 2, where the tail skips nothing, each tier + a fifth of the tail's 1e-12), recomputing
    any tile over it exactly.  On EVERY ion, against the same engine with the
    tail and every form off: |dF_i| <= the measured bound of that call (force_tail_bound, the largest
    per-sub-tile sum after the exact pass) + the summation-order rounding, for the defaults and each
    tier alone; the measured bound <= force_error_eps; on these uniform configurations no tile over it"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS[cfg]).init()
    L = s.const("L")
    assert s.const("force_form_mode") == 2 and s.const("force_form_measured") == 1
    tiers = ("mid", "far", "vfar", "ufar", "ufar32")
    r2, e2 = {k: s.const(f"force_{k}_radius") for k in tiers}, s.const("force_error_eps")
    s.set_option("force_form_mode", 0)
    r0 = {k: s.const(f"force_{k}_radius") for k in tiers}
    s.set_option("force_form_mode", 1)
    r1, e1 = {k: s.const(f"force_{k}_radius") for k in tiers}, s.const("force_error_eps")
    print(f"{cfg}: radii form mode 1 {dict((k, round(v, 3)) for k, v in r1.items())}, mode 2 "
          f"{dict((k, round(v, 3)) for k, v in r2.items())}, mode 0 {dict((k, round(v, 3)) for k, v in r0.items())}, "
          f"L/2 {L / 2:.3f}; force_error_eps mode 1 {e1:.2e}, mode 2 {e2:.2e}")
    assert r1["mid"] < r1["far"] < r1["vfar"] <= r1["ufar"] <= r1["ufar32"] <= L / 2
    for k in ("mid", "far", "vfar", "ufar"):
        assert r1[k] < r0[k]
    # mode 2: where the tail skips nothing (C5) the tiers share its 1e-12 — one total per ion, 1.5e-12
    if s.const("force_skip_radius") >= L / 2:
        assert e2 == pytest.approx(1.5e-12, rel=1e-12) and e1 == pytest.approx(5e-13, rel=1e-12)
        assert all(r2[k] <= r1[k] for k in tiers) and r2["far"] < r1["far"]
    else:
        assert e2 == e1 and r2 == r1
    s.set_option("force_form_mode", 2)
    out, tb, eps = {}, {}, {}
    combos = ((12, 13, 13, 13, 13), (0, 13, 0, 0, 0), (0, 0, 13, 0, 0), (0, 0, 0, 13, 0), (0, 0, 0, 0, 13),
              (0, 0, 0, 0, 0))
    for key in combos:
        for o, v in zip(("force_tail_exp", "force_mid_exp", "force_far_exp", "force_vfar_exp", "force_ufar_exp"), key):
            s.set_option(o, v)
        s.forces()
        out[key] = s.get_state()["F"]
        tb[key], eps[key] = s.const("force_tail_bound"), s.const("force_error_eps")
        assert s.const("force_tail_fixed_tiles") == 0
    Fe = out[0, 0, 0, 0, 0]
    assert eps[0, 0, 0, 0, 0] == 0 and tb[0, 0, 0, 0, 0] == 0      # (nothing approximate: nothing measured)
    scale = 1e-13 * np.abs(Fe).max()
    for key in combos[:-1]:
        d = np.abs(out[key] - Fe).max()
        print(f"{cfg} {key}: max_i |dF_i| {d:.3e}, measured bound {tb[key]:.3e}, eps {eps[key]:.2e}")
        assert 0 < tb[key] <= eps[key]
        assert d <= tb[key] + scale
    s.close()


def clustered_state(N0, L, frac, rc, seed=5):
    """A deliberately clustered configuration: a fraction `frac` of the N0 ions uniform in a ball of
    radius rc at the box centre, the rest uniform in the box, in random index order — far from the
    uniform density the skip radius's model (mdqt_engine.cpp tail_radius_sum) assumes.  V = 0,
    every psi = |0>, tPart = 0, t = 0."""
    rng = np.random.default_rng(seed)
    nc = int(frac * N0)
    u = rng.normal(size=(3, nc))
    u /= np.linalg.norm(u, axis=0)
    ball = L / 2 + u * (rc * rng.uniform(0, 1, nc) ** (1 / 3))
    R = np.concatenate([rng.uniform(0, L, (3, N0 - nc)), ball], axis=1)[:, rng.permutation(N0)]
    R = np.ascontiguousarray(R)
    psi = np.zeros((N0, 12, 2))
    psi[:, 0, 0] = 1.0
    return R, np.zeros((3, N0)), psi, np.zeros(N0), 0.0


# (N0, force_tail_exp, cluster fraction, cluster radius): N0 = 70,000 with eps = 1e-4 puts the skip
# radius inside L/2 at a size that runs in seconds; N = 1e6 is north_star's size at the product
# default eps = 1e-12
CLUSTERED = {"70k": (70000, 4, 0.5, 2.0), "1M": (1000000, 12, 0.2, 12.0)}


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["70k", "1M"])
def test_tail_bound_enforced_on_clustered_ions(cfg, orc):
    """force_tail_mode 1 on a configuration the density model gets wrong: a dense ball of ions.
    The skip radius r_t the model picks leaves some tiles with a tail sum over eps; the engine must
    catch it — k_tail_fix recomputes those tiles' forces exactly, so EVERY ion's force stays within
    eps of the exact sum to L/2 (SpeedUp:195, :222), and at the next sync the host widens r_t.
    Checked on every ion against the same engine with the tail and the far forms off (the exact
    pair form on every pair inside L/2): tail alone within eps, the product defaults within eps +
    the far forms' bounds, each + the rounding of the sums (below: 1e-15 of the ion's partial-sum
    scale, sharp on most ions)."""
    import mdqtplasmasims_amd as M
    N0, k, frac, rc = CLUSTERED[cfg]
    eps = 10.0 ** -k
    s = M.Simulation(N0=N0, seed=SEED, job=1, rng_mode=1)
    L = s.const("L")
    state = clustered_state(N0, L, frac, rc)
    s.set_state(*state)
    s.set_option("force_tail_exp", k)
    assert s.const("force_scheme") == 3 and s.const("force_tail_mode") == 1
    rt0 = s.const("force_skip_radius")
    assert rt0 < L / 2
    fb = (s.const("force_far_bound") + s.const("force_vfar_bound") + s.const("force_ufar_bound")
          + s.const("force_mid_bound"))
    # force_form_mode 1: the sums hold the forms' terms too, held to force_error_eps (eps + the tiers')
    ea = s.const("force_error_eps") if s.const("force_form_measured") else eps
    fb = max(fb, ea - eps)
    out = {}
    # A: the product defaults; the model's r_t is too small here
    s.forces()
    out["A"] = s.get_state()["F"]                        # (a sync: the host reacts)
    fixed, raw, tb = s.const("force_tail_fixed_tiles"), s.const("force_tail_raw_bound"), s.const("force_tail_bound")
    scale, rt1 = s.const("force_tail_scale"), s.const("force_skip_radius")
    print(f"{cfg}: N={s.N} L/2={L / 2:.3f} eps={eps:.0e}: model r_t {rt0:.3f}; tiles over eps {fixed:.0f}, largest "
          f"per-tile sum {raw:.3e}, bound met after the exact pass {tb:.3e}; r_t widened to {rt1:.3f} (scale {scale:.2f})")
    assert fixed > 0 and raw > ea                       # the model radius was too small: caught
    assert tb <= ea                                      # and enforced
    assert scale > 1 and rt0 < rt1 <= L / 2              # widened for the calls to come
    # B: the next call at the widened radius
    s.forces()
    out["B"] = s.get_state()["F"]
    fixed_b = s.const("force_tail_fixed_tiles") - fixed
    print(f"{cfg}: at r_t {rt1:.3f}: tiles over eps {fixed_b:.0f}, bound {s.const('force_tail_bound'):.3e}")
    assert s.const("force_tail_bound") <= ea
    # new positions of the same system keep the widened radius (a driver that uploads R every MD step
    # does not rerun the exact pass at every call)
    s.set_state(*state)
    assert s.const("force_skip_radius") == rt1
    # C: the tail alone (far forms off), from the model's radius again (a tail option resets the scale)
    s.set_option("force_tail_mode", 0)
    s.set_option("force_tail_mode", 1)
    for o in ("force_mid_exp", "force_far_exp", "force_vfar_exp", "force_ufar_exp"):
        s.set_option(o, 0)
    assert s.const("force_skip_radius") == rt0
    s.forces()
    out["C"] = s.get_state()["F"]
    assert s.const("force_tail_fixed_tiles") > 0 and s.const("force_tail_bound") <= eps
    # E: exact — no skip radius, no far forms
    s.set_option("force_tail_exp", 0)
    assert s.const("force_skip_radius") == L / 2
    s.forces()
    Fe = s.get_state()["F"]
    lD = s.const("lDeb")
    s.close()
    # The sums' rounding: C and E sum the same terms but for the dropped ones, in the block kernel's
    # order (the dropped terms move the partial sums' roundings) or, on the tiles k_tail_fix
    # recomputed, in its order (compensated: within a few ulp of |F_i|).  Their difference is a few
    # ulp of the ion's largest partial sums, which in the ball (ions ~0.3 apart, |F| ~ 4e3) exceed
    # 1e-12 / u: scale P_i = max(|F_i|, the sum of its 16 nearest neighbours' pair terms g(r))
    # (periodic KD tree), allowed as 1e-15 P_i (~9 u P_i).  Where that is below eps / 10 the check is
    # sharp (most ions; measured worst |dF_i| 4.6e-13 there, ions ~r_t from the ball).
    from scipy.spatial import cKDTree
    R = state[0]
    r = cKDTree(R.T, boxsize=L).query(R.T, k=17)[0][:, 1:]
    P = np.maximum(np.abs(Fe).max(axis=0), ((1 / r + 1 / lD) * np.exp(-r / lD) / r).sum(axis=1))
    rnd = 1e-15 * P
    d = {key: np.abs(v - Fe).max(axis=0) for key, v in out.items()}
    sharp = rnd < eps / 10
    print(f"{cfg}: max|F| {np.abs(Fe).max():.3e}; max_i |dF_i|: defaults {d['A'].max():.3e} (after widening "
          f"{d['B'].max():.3e}), tail only {d['C'].max():.3e}; far bounds {fb:.2e}; sharp check on "
          f"{sharp.mean():.1%} of the ions (tail only there: max {d['C'][sharp].max():.3e})")
    assert sharp.mean() > 0.5
    assert np.all(d["C"] <= eps + rnd)
    assert np.all(d["A"] <= eps + fb + rnd) and np.all(d["B"] <= eps + fb + rnd)
    # the ions where that check is not sharp (the ball: the exact pass's tiles), against the oracle's
    # compensated rows instead of the engine's exact mode, so that only A's own rounding is allowed
    # (ADVICE r04): within eps + the far bounds + 1e-15 P_i of the compensated sum
    loose = np.flatnonzero(~sharp)
    if not len(loose):                                  # (eps 1e-4 at 70k: every ion's check is sharp)
        return
    idx = np.sort(np.random.default_rng(7).choice(loose, min(256, len(loose)), replace=False))
    G = orc.forces_index(R, idx, L, lD, nthreads=threads())
    dA = np.abs(out["A"][:, idx] - G).max(axis=0)
    print(f"{cfg}: {len(idx)} of the {len(loose)} ball ions against the compensated oracle: max |dF_i| {dA.max():.3e}, "
          f"max |dF_i| / P_i {(dA / P[idx]).max():.2e}")
    assert np.all(dA <= eps + fb + rnd[idx])


@pytest.mark.gpu
def test_form_bound_enforced_on_clustered_ions():
    """force_form_mode 1 on a configuration its density model gets wrong (round 6): the 70k clustered
    state with the tail off, so the sums hold the error-bounded forms' terms alone — the ions around the
    ball see ~35,000 ions at the mid / far radii, far more than the model's uniform density.  The first
    call must list the tiles whose sums exceed force_error_eps and recompute them exactly (k_tail_fix),
    the host widens the model (force_tail_scale; every tier radius grows), and EVERY ion's force is
    within force_error_eps of the exact sum to L/2 (the engine with every form off) + the rounding of
    the sums (as in test_tail_bound_enforced_on_clustered_ions)"""
    import mdqtplasmasims_amd as M
    N0, _, frac, rc = CLUSTERED["70k"]
    s = M.Simulation(N0=N0, seed=SEED, job=1, rng_mode=1)
    L = s.const("L")
    state = clustered_state(N0, L, frac, rc)
    s.set_state(*state)
    s.set_option("force_tail_exp", 0)
    assert s.const("force_form_measured") == 1 and s.const("force_skip_radius") == L / 2
    ea = s.const("force_error_eps")
    rad0 = {k: s.const(f"force_{k}_radius") for k in ("mid", "far", "vfar", "ufar")}
    assert ea > 0 and rad0["mid"] < L / 2
    s.forces()
    FA = s.get_state()["F"]                             # (a sync: the host reacts)
    fixed, raw, tb = s.const("force_tail_fixed_tiles"), s.const("force_tail_raw_bound"), s.const("force_tail_bound")
    rad1 = {k: s.const(f"force_{k}_radius") for k in ("mid", "far", "vfar", "ufar")}
    print(f"70k clustered, forms only: eps {ea:.2e}; tiles over it {fixed:.0f}, largest sum {raw:.3e}, bound after "
          f"the exact pass {tb:.3e}; radii {rad0} -> {rad1} (scale {s.const('force_tail_scale'):.0f})")
    assert fixed > 0 and raw > ea and tb <= ea
    assert s.const("force_tail_scale") > 1 and all(rad1[k] > rad0[k] for k in rad0 if rad0[k] < L / 2)
    s.forces()
    FB = s.get_state()["F"]
    assert s.const("force_tail_bound") <= ea
    for o in ("force_mid_exp", "force_far_exp", "force_vfar_exp", "force_ufar_exp"):
        s.set_option(o, 0)
    s.forces()
    Fe = s.get_state()["F"]
    lD = s.const("lDeb")
    s.close()
    from scipy.spatial import cKDTree
    R = state[0]
    r = cKDTree(R.T, boxsize=L).query(R.T, k=17)[0][:, 1:]
    P = np.maximum(np.abs(Fe).max(axis=0), ((1 / r + 1 / lD) * np.exp(-r / lD) / r).sum(axis=1))
    rnd = 1e-15 * P
    dA, dB = np.abs(FA - Fe).max(axis=0), np.abs(FB - Fe).max(axis=0)
    sharp = rnd < ea / 10
    print(f"70k clustered, forms only: max_i |dF_i| first call {dA.max():.3e}, after widening {dB.max():.3e}; "
          f"sharp check on {sharp.mean():.1%} of the ions (there: {dA[sharp].max():.3e}); elsewhere max |dF_i| / "
          f"(eps + 1e-15 P_i) {(dA / (ea + rnd)).max():.3f}")
    assert sharp.mean() > 0.4                            # (the ball's half of the ions: rounding-scale sums)
    assert np.all(dA <= ea + rnd) and np.all(dB <= ea + rnd)


@pytest.mark.gpu
def test_tail_bound_enforced_in_sharded_local_group():
    """The measured, enforced tail at world > 1: the ranks' per-tile sums are
    summed before the enforcement (ncclAllReduce in a real group; in-process here, one MI355X), so
    world 2 flags the same tiles as world 1 and agrees with it within the rank-order rounding"""
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_init_local
    N0, k, frac, rc = CLUSTERED["70k"]
    ref = M.Simulation(N0=N0, seed=SEED, rng_mode=1)
    state = clustered_state(N0, ref.const("L"), frac, rc)
    ref.set_state(*state)
    ref.set_option("force_tail_exp", k)
    sims = [M.Simulation(N0=N0, seed=SEED, rng_mode=1, world_size=2, rank=r) for r in range(2)]
    for x in sims:
        x.set_state(*state)
        x.set_option("force_tail_exp", k)
        assert x.const("force_scheme") == 3 and x.const("force_skip_radius") == ref.const("force_skip_radius")
    comm_init_local(sims)
    for x in sims:
        x.allgather_positions()
    for x in sims:
        x.forces()
    ref.forces()
    G = ref.get_state()["F"]
    worst = 0.0
    for x in sims:
        lo, hi = x.slab_bounds()
        worst = max(worst, np.abs(x.get_state()["F"][:, lo:hi] - G[:, lo:hi]).max() / np.abs(G).max())
    counts = [x.const("force_tail_fixed_tiles") for x in sims]
    print(f"world 2 vs 1: max|dF|/max|F| = {worst:.3e}; tiles over eps {counts} vs {ref.const('force_tail_fixed_tiles'):.0f}; "
          f"r_t {[x.const('force_skip_radius') for x in sims]} vs {ref.const('force_skip_radius'):.3f}")
    assert worst < 1e-13
    assert counts[0] == counts[1] == ref.const("force_tail_fixed_tiles") > 0
    assert sims[0].const("force_skip_radius") == sims[1].const("force_skip_radius") == ref.const("force_skip_radius")
    for x in sims:
        x.close()
    ref.close()


@pytest.mark.gpu
def test_tail_option_change_between_forces_and_reduce():
    """a tail option changed on one rank of an in-process group after forces() and before
    the deferred reduce must not drop the enforcement — set_option settles the pending partials first
    (with the eps they were measured for), so both ranks still match world 1"""
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_init_local
    N0, k, frac, rc = CLUSTERED["70k"]
    ref = M.Simulation(N0=N0, seed=SEED, rng_mode=1)
    state = clustered_state(N0, ref.const("L"), frac, rc)
    ref.set_state(*state)
    ref.set_option("force_tail_exp", k)
    ref.forces()
    G = ref.get_state()["F"]
    assert ref.const("force_tail_fixed_tiles") > 0
    sims = [M.Simulation(N0=N0, seed=SEED, rng_mode=1, world_size=2, rank=r) for r in range(2)]
    for x in sims:
        x.set_state(*state)
        x.set_option("force_tail_exp", k)
    comm_init_local(sims)
    for x in sims:
        x.allgather_positions()
    for x in sims:
        x.forces()
    sims[0].set_option("force_tail_exp", k + 1)        # between forces() and the reduce
    worst = 0.0
    for x in sims:
        lo, hi = x.slab_bounds()
        worst = max(worst, np.abs(x.get_state()["F"][:, lo:hi] - G[:, lo:hi]).max() / np.abs(G).max())
    print(f"tail option changed before the reduce: world 2 vs 1 max|dF|/max|F| = {worst:.3e}")
    assert worst < 1e-13
    for x in sims:
        x.close()
    ref.close()


def _tiny_state(x):
    """a state of N = N0 ions (uniform positions) without init()'s sampling, for constant checks"""
    N = int(x.params.N0)
    rng = np.random.default_rng(0)
    L = x.const("L")
    psi = np.zeros((N, 12, 2)); psi[:, 0, 0] = 1.0
    return rng.uniform(0, L, (3, N)), np.zeros((3, N)), psi, np.zeros(N), 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_newton3_blocks_above_64k_local_group(world, orc):
    """N > 65,536 (Newton-3 blocks in Hilbert order, the scheme every sharded BASELINE config uses)
    as an in-process rank group on one MI355X: each rank evaluates its blocks' pairs for all ions,
    the dense partials are summed in rank order (RCCL's reduce-scatter in a real group).  Stated
    cross-world tolerance: forces within 1e-13 of world 1 (max-norm relative), positions and
    velocities within 1e-12 after two MD steps with QT on (the rank-order sum changes rounding only)"""
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_init_local
    kw = dict(N0=70000, seed=19, rng_mode=1)
    ref = M.Simulation(**kw).init()
    assert ref.const("force_scheme") == 3 and ref.N > 65536
    st = ref.get_state()
    sims = [M.Simulation(world_size=world, rank=r, **kw) for r in range(world)]
    for s in sims:
        s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
        assert s.const("force_scheme") == 3
    comm_init_local(sims)
    for s in sims:
        s.allgather_positions()
    for s in sims:
        s.forces()
    ref.forces()
    G = ref.get_state()["F"]
    worst = 0.0
    for s in sims:
        lo, hi = s.slab_bounds()
        F = s.get_state()["F"][:, lo:hi]
        worst = max(worst, np.abs(F - G[:, lo:hi]).max() / np.abs(G).max())
    print(f"world {world}: forces vs world 1 max|dF|/max|F| = {worst:.3e}")
    assert worst < 1e-13
    ratio = int(ref.const("plasmaToQuantumTimestepRatio"))
    for _ in range(2):
        for s in sims:
            s.substeps(ratio)
        for s in sims:
            s.allgather_positions()
        for s in sims:
            s.forces()
    for s in sims:
        s.substeps(ratio)
    ref.substeps(ratio)
    ref.md_steps(2)
    b = ref.get_state()
    for s in sims:
        lo, hi = s.slab_bounds()
        a = s.get_state()
        dR = np.abs(a["R"][:, lo:hi] - b["R"][:, lo:hi]).max()
        dV = np.abs(a["V"][:, lo:hi] - b["V"][:, lo:hi]).max()
        assert dR < 1e-12 and dV < 1e-12, (dR, dV)
    for s in sims:
        s.close()
    ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sort", [1, 0])
def test_epotential_newton3_blocks_match_rows(sort):
    """Epotential() above 65,536 ions on the Newton-3 blocks (the block kernel's POT mode, world 1,
    Hilbert order with tile-pair skipping or storage order) against the owner-computes rows"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(N0=70000, seed=23, rng_mode=1).init()
    s.set_option("force_sort", sort)
    s.md_steps(1)
    assert s.const("force_scheme") == 3 and s.const("potential_n3") == 1
    e3 = s.Epotential()
    s.set_option("potential_n3", 0)
    er = s.Epotential()
    s.close()
    print(f"N0=70000 sort={sort}: Epot blocks {e3:.15e} rows {er:.15e}")
    assert abs(e3 - er) <= 1e-13 * abs(er), (e3, er)


@pytest.mark.gpu
def test_raw_rsq_error_within_the_very_far_bound():
    """The very-far pair form's bound assumes v_rsq_f64 is within kRsqRawErr = 2^-23 of 1/sqrt(x)
    (mdqt_internal.hpp): tools/rsq_precision (built by __graft_entry__.build()) measures it on 4M
    inputs over r^2 in [1e-4, 1e6] against a long-double reference"""
    import re
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "rsq_precision")
    assert os.path.exists(exe), "tools/rsq_precision missing: run __graft_entry__.build()"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120).stdout
    raw = float(re.search(r"raw ([0-9.e+-]+)", out).group(1))
    f32 = float(re.search(r"rsq_f32: ([0-9.e+-]+)", out).group(1))
    print(out.strip())
    assert raw <= 2.0 ** -23
    assert f32 <= 2.0 ** -23                         # kRsqF32RelErr: the f32 ultra-far form's bound


@pytest.mark.gpu
def test_exp2f_error_within_the_ultra_far_bound():
    """The ultra-far pair form's bound assumes v_exp_f32 is within kExp2fRelErr = 2^-22 of 2^x
    (mdqt_internal.hpp): tools/exp2f_precision measures it on 16M inputs over x in [-70, 0]"""
    import re
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "exp2f_precision")
    assert os.path.exists(exe), "tools/exp2f_precision missing: run __graft_entry__.build()"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120).stdout
    err = float(re.search(r"exp2f: ([0-9.e+-]+)", out).group(1))
    print(out.strip())
    assert err <= 2.0 ** -22


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_masked_reduction_bit_identical(world):
    """k_n3b_reduce with the plan's per-J-tile masks (force_reduce_mask 1, the default) reads only the
    j-slots the block kernel wrote and skips the -0 of empty J steps: F bit for bit the same as reading
    every slot (option 0), at world 1 and in a world-2 in-process group (N0 = 250,000: the tail radius
    and the ultra-far tiers leave ~2/3 of the J steps empty at the far block distances)"""
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_init_local
    kw = dict(N0=250000, detuningDP=1.0, seed=SEED, job=1)
    ref = M.Simulation(**kw).init()
    st = ref.get_state()
    ref.close()
    out = {}
    for mode in (1, 0):
        sims = [M.Simulation(world_size=world, rank=r, **kw) for r in range(world)]
        for s in sims:
            s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
            s.set_option("force_reduce_mask", mode)
            assert s.const("force_reduce_mask") == mode
        if world > 1:
            comm_init_local(sims)
            for s in sims:
                s.allgather_positions()
        for s in sims:
            s.forces()
        F = np.zeros_like(st["R"])
        for s in sims:
            lo, hi = s.slab_bounds()
            F[:, lo:hi] = s.get_state()["F"][:, lo:hi]
        for s in sims:                                  # (after every rank's reduce: they share partials)
            s.close()
        out[mode] = F
    assert np.array_equal(out[1], out[0])


@pytest.mark.gpu
def test_block_work_sums_to_the_census():
    """mdqt_force_block_work (the load-balance census): one entry per block, summing to the census's
    evaluated lane-steps; at world 2 each rank's blocks are its half of the world-1 array"""
    import mdqtplasmasims_amd as M
    kw = dict(N0=100000, Ge=1.0 / 12, qt_enabled=0, seed=SEED, job=1)
    s = M.Simulation(**kw).init()
    w = s.force_block_work()
    cen = s.force_census()
    ev = sum(v[0] for k, v in cen.items() if not k.startswith("skip"))
    assert len(w) == int(s.const("n3b_block_count")) and w.min() > 0
    assert w.sum() == ev
    NB = len(w)
    print(f"C3 blocks {NB}: per-block evaluated lane-steps min/mean/max {w.min() / w.mean():.3f} / 1 / "
          f"{w.max() / w.mean():.3f}; world-8 partition max/mean "
          f"{max(w[r * NB // 8:(r + 1) * NB // 8].sum() for r in range(8)) / (w.sum() / 8):.4f}")
    s.close()


@pytest.mark.gpu
def test_weighted_block_ranges_local_group():
    """force_balance 1 (default): the sharded ranks' block ranges by the census's work (n3b_balance) —
    a partition of all blocks, the same on every rank, no rank's work above the equal-count split's
    worst, and the forces still world 1's within 1e-13"""
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_init_local
    kw = dict(N0=250000, detuningDP=1.0, seed=SEED, job=1)
    ref = M.Simulation(**kw).init()
    st = ref.get_state()
    ref.forces()
    G = ref.get_state()["F"]
    NB = int(ref.const("n3b_block_count"))
    ref.close()
    W = 4
    sims = [M.Simulation(world_size=W, rank=r, **kw) for r in range(W)]
    for s in sims:
        s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    comm_init_local(sims)
    for s in sims:
        s.allgather_positions()
    for s in sims:
        s.forces()
    ranges = [(int(s.const("n3b_block_lo")), int(s.const("n3b_block_hi"))) for s in sims]
    assert ranges[0][0] == 0 and ranges[-1][1] == NB
    assert all(ranges[r][1] == ranges[r + 1][0] for r in range(W - 1))
    ratios = {(s.const("force_balance_ratio"), s.const("force_balance_ratio_equal")) for s in sims}
    assert len(ratios) == 1                              # every rank computed the same partition
    wr, er = ratios.pop()
    print(f"C5 world {W}: weighted ranges {ranges}; max/mean work {wr:.4f} (equal counts {er:.4f})")
    assert wr <= er + 1e-12 and wr < 1.02
    worst = 0.0
    for s in sims:
        lo, hi = s.slab_bounds()
        worst = max(worst, np.abs(s.get_state()["F"][:, lo:hi] - G[:, lo:hi]).max() / np.abs(G).max())
    assert worst < 1e-13
    for s in sims:
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C3", "C5", "C4", "1M"])
def test_epotential_on_the_plan(cfg, orc):
    """Epotential() (SpeedUp:244-281) on the Newton-3 blocks with the force call's plan (round 6, VERDICT
    r05 item 2; option potential_plan 1): skip radius, sub-tile groups, the error-bounded pair forms for
    u = e^(-r/lDeb)/r and the enforced tail.  Since u(r) < lDeb g(r) and each form's relative error on u is
    at most its error on the force, every U_i stays within lDeb x (the tail eps 1e-12 + the tiers' bounds;
    force_form_mode 1: the eps the call's measured sums are held to, force_error_eps) of the sum to L/2 — checked on ~640 sampled ions against the oracle's compensated rows
    (orc_potentials_index), beside the exact block path (potential_plan 0); Epot = sum U_i / 2N within
    1e-12 relative of the exact path's (north_star asks 1e-6 relative for energies)"""
    import mdqtplasmasims_amd as M
    if M.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked tests")
    kw = dict(CONFIGS[cfg])
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **kw).init()
    N, L, lDeb = s.N, s.const("L"), s.const("lDeb")
    assert s.const("force_scheme") == 3 and s.const("potential_plan") == 1
    U1 = s.potential_rows()
    e1 = s.Epotential()
    s.set_option("potential_plan", 0)
    U0 = s.potential_rows()
    e0 = s.Epotential()
    R = s.get_state()["R"]
    bounds = sum(s.const(k) for k in ("force_mid_bound", "force_far_bound", "force_vfar_bound", "force_ufar_bound"))
    # force_form_mode 1: the force sums are held to force_error_eps (tail + tiers, measured and enforced)
    per_ion = max(1e-12 + bounds, s.const("force_error_eps"))
    s.close()
    rng = np.random.default_rng(5)
    idx = sample_ions(N, 640, rng)
    G = orc.potentials_index(R, idx, L, lDeb, nthreads=threads())
    d1, d0 = np.abs(U1[idx] - G).max(), np.abs(U0[idx] - G).max()
    gate = lDeb * per_ion + 1e-13 * np.abs(G).max()
    rel = abs(e1 - e0) / abs(e0)
    print(f"{cfg}: N={N} sampled {len(idx)}: plan max|dU| = {d1:.3e} (gate {gate:.3e}), exact max|dU| = {d0:.3e}; "
          f"Epot plan {e1:.15g} exact {e0:.15g} rel {rel:.2e}; max|U_plan - U_exact| over all ions "
          f"{np.abs(U1 - U0).max():.3e}")
    assert d0 <= 1e-12 * np.abs(G).max()
    assert d1 <= gate
    assert np.abs(U1 - U0).max() <= gate + 1e-13 * np.abs(U0).max()
    assert rel <= 1e-12
    assert abs(e1 - U1.sum() / 2 / N) <= 1e-12 * abs(e1)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C3", "1M"])
def test_paired_wave_kernel_matches_eight_wave_kernel(cfg):
    """force_n3b_pairs (round 6): the paired-wave block kernel (k_pairs_n3b_pw: 4 waves, two I tiles each,
    paired per block distance by the plan) against the 8-wave kernel on the same plan — the same pair
    terms in another j-side summation order: within rounding (1e-13 of max |F|), momentum conserved; and
    the pairing is a function of the positions: two calls give the same bits"""
    import mdqtplasmasims_amd as M
    s = M.Simulation(seed=SEED, job=1, rng_mode=1, **CONFIGS[cfg]).init()
    assert s.const("force_n3b_pairs") == 1
    out = {}
    for mode in (1, 0):
        s.set_option("force_n3b_pairs", mode)
        s.forces()
        out[mode] = s.get_state()["F"]
    s.set_option("force_n3b_pairs", 1)
    s.forces()
    again = s.get_state()["F"]
    N = s.N
    s.close()
    scale = np.abs(out[0]).max()
    err = np.abs(out[1] - out[0]).max() / scale
    mom = np.abs(out[1].sum(axis=1)).max() / (np.abs(out[1]).sum() / N)
    print(f"{cfg}: paired vs 8-wave block kernel max|dF|/max|F| = {err:.3e}, |sum F| / mean|F| = {mom:.3e}")
    assert err <= 1e-13
    assert mom <= 1e-9
    assert np.array_equal(again, out[1])
