"""force_form_mode 1's tier radii (round 6; mdqt_engine.cpp model_tier_radius, exported as
mdqt_tier_radius_model — host arithmetic, no device): against a numpy restatement of the density model,
against the radii the GPU runs reported (profiles/r06f_form_census.txt), and the invariants the
enforcement relies on (the model radius never beyond the a-priori cap, the tiers in order, wider with a
larger model scale or a smaller eps)."""
import math

import numpy as np
import pytest

from mdqtplasmasims_amd.engine import tier_radius_model

# far_err's constants (mdqt_internal.hpp)
K_RSQ1, K_TAB4, K_FAR = 2.2e-14, 4e-15, 3e-9
K_RAW, K_EXP5, K_EXP2F = 2.0 ** -23, 1.1e-7, 2.0 ** -22
K_U32A, K_U32B = 22 * 2.0 ** -24, 52 * 2.0 ** -24
LEVELS = {"mid": 5, "far": 1, "vfar": 2, "ufar": 3, "ufar32": 4}


def g(r, l):
    return (1 / r + 1 / l) * np.exp(-r / l) / r


def err(r, l, lv):
    if lv == 5:
        return (r / l + 3) * (K_RSQ1 + 2.0 ** -52) + K_TAB4
    if lv == 4:
        return (r / l) * K_U32A + K_U32B
    if lv == 3:
        return (r / l) * (K_RAW + 2.0 ** -24) + 3 * K_RAW + K_EXP2F
    if lv == 2:
        return (r / l + 3) * K_RAW + K_EXP5
    return K_FAR


def model(r, hi, N, L, l, lv):
    """rho int_r^hi 4 pi (x + delta)^2 g(x) err(x) dx, delta two 16-ion sub-tile widths (Simpson, 2000)"""
    rho = N / L ** 3
    d = 2 * (16 / rho) ** (1 / 3)
    if r >= hi:
        return 0.0
    x = np.linspace(r, hi, 2001)
    y = 4 * np.pi * (x + d) ** 2 * g(x, l) * err(x, l, lv)
    w = np.ones(2001)
    w[1:-1:2], w[2:-1:2] = 4, 2
    return rho * (w * y).sum() * (hi - r) / 2000 / 3


def model_radius(N, L, l, k, lv, hi, scale=1.0):
    lo, up = 0.0, hi
    for _ in range(60):
        if up - lo <= 1e-9 * L / 2:
            break
        m = 0.5 * (lo + up)
        if m > 0 and 1.25 * scale * model(m, hi, N, L, l, lv) <= 10.0 ** -k:
            up = m
        else:
            lo = m
    return up


def box(N0):
    return (N0 * 4 * math.pi / 3) ** 0.333333333      # SpeedUp:297


# (N0, N, lDeb, skip radius r_t) of the GPU runs and the radii they reported (profiles/r06f_form_census.txt)
RUNS = {
    "C5": (250000, 249970, 1 / math.sqrt(0.3), None,
           {"mid": 10.56, "far": 28.44, "vfar": 41.59, "ufar": 42.33, "ufar32": 46.0}),
    "C4": (1000000, 1000258, 2.0, 66.871,
           {"mid": 11.62, "far": 31.26, "vfar": 45.72, "ufar": 46.54, "ufar32": 50.72}),
    "1M": (1000000, 1000258, 1 / math.sqrt(0.3), 60.914,
           {"mid": 10.56, "far": 28.44, "vfar": 41.61, "ufar": 42.36, "ufar32": 46.17}),
}


@pytest.mark.parametrize("cfg", sorted(RUNS))
def test_model_radii_match_gpu_runs_and_restatement(cfg):
    N0, N, l, rt, ref = RUNS[cfg]
    L = box(N0)
    hi = L / 2 if rt is None else rt
    for name, lv in LEVELS.items():
        r, b = tier_radius_model(N, L, l, 13, lv, hi)
        assert abs(r - ref[name]) <= 0.006, (cfg, name, r, ref[name])
        rn = model_radius(N, L, l, 13, lv, hi)
        assert abs(r - rn) <= 1e-6 * L, (cfg, name, r, rn)
        assert 0 < b <= 1e-13 / 1.25 * (1 + 1e-9)
        assert abs(b - model(r, hi, N, L, l, lv)) <= 1e-6 * b


@pytest.mark.parametrize("cfg", sorted(RUNS))
def test_model_radius_invariants(cfg):
    N0, N, l, rt, _ = RUNS[cfg]
    L = box(N0)
    hi = L / 2 if rt is None else rt
    rad = {name: tier_radius_model(N, L, l, 13, lv, hi)[0] for name, lv in LEVELS.items()}
    assert rad["mid"] < rad["far"] < rad["vfar"] <= rad["ufar"] <= rad["ufar32"] <= L / 2
    for name, lv in LEVELS.items():
        r = rad[name]
        cap = tier_radius_model(N, L, l, 13, lv, hi, apriori=2)[0]
        mode0 = tier_radius_model(N, L, l, 13, lv, hi, apriori=1)[0]
        assert r <= cap <= mode0                       # the a-priori radius bounds any configuration
        assert r < mode0                               # and the model is what makes the difference here
        # a configuration over its bound doubles the model's scale: every radius widens
        assert tier_radius_model(N, L, l, 13, lv, hi, scale=2.0)[0] > r
        # a tighter eps moves the tier out
        assert tier_radius_model(N, L, l, 14, lv, hi)[0] > r
    # k = 0: the tier off (L/2, bound 0)
    assert tier_radius_model(N, L, l, 0, 1, hi) == (L / 2, 0.0)


def test_model_radius_rejects_bad_arguments():
    from mdqtplasmasims_amd import MdqtError
    with pytest.raises(MdqtError):
        tier_radius_model(1000, 20.0, 1.8, 13, 6, 10.0)
    with pytest.raises(MdqtError):
        tier_radius_model(1000, 20.0, 1.8, 13, 1, 10.0, apriori=3)
