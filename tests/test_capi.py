"""CPU checks of the drop-in boundary (no GPU needed): libmdqt.so builds, loads, exports every
symbol include/mdqt.h declares, the Python mirror binds all of them, the pure host functions
behave, and the product path fails loudly (never silently falls back) without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mdqt.h")


@pytest.fixture(scope="module")
def L():
    from mdqtplasmasims_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from mdqtplasmasims_amd.build import build
        build(quiet=True)
    return _lib.lib()


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mdqt_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_the_seam():
    syms = header_symbols()
    for s in ("mdqt_forces", "mdqt_step", "mdqt_qstep", "mdqt_substeps", "mdqt_init", "mdqt_output",
              "mdqt_write_conditions", "mdqt_read_conditions", "mdqt_run", "mdqt_epotential"):
        assert s in syms


def test_library_exports_every_header_symbol(L):
    missing = [s for s in header_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_python_binding_covers_header(L):
    from mdqtplasmasims_amd._lib import SIGNATURES
    bound = {s[0] for s in SIGNATURES}
    assert set(header_symbols()) == bound


def test_default_params_are_the_reference_defaults(L, orc):
    from mdqtplasmasims_amd.engine import default_params
    p = default_params()
    o = orc.default_params()
    for k in ("Ge", "tmax", "density", "sig0", "Te", "fracOfSig", "detuning", "detuningDP", "Om", "OmDP",
              "N0", "newRun", "c0", "sampleFreq", "reNormalizewvFns"):
        assert getattr(p, k) == getattr(o, k), k
    # SpeedUp:60-78
    assert (p.Ge, p.tmax, p.density, p.N0, p.sampleFreq) == (0.1, 30, 2, 3500, 40)
    assert p.saveDirectory == b"dataLaserCool/"


def test_params_struct_layout_matches_header(L):
    from mdqtplasmasims_amd._lib import MdqtParams
    src = open(HEADER).read()
    body = src[src.index("typedef struct mdqt_params {"):src.index("} mdqt_params;")]
    names = re.findall(r"\b(?:double|int|uint32_t|char)\s+(\w+)", body)
    assert names == [f[0] for f in MdqtParams._fields_]


@pytest.mark.parametrize("N,world", [(0, 1), (1, 1), (3573, 1), (3573, 2), (1000, 8), (1000000, 8), (250000, 3)])
def test_slab_partition(L, N, world):
    from mdqtplasmasims_amd.engine import slab
    covered = []
    S0 = None
    for r in range(world):
        lo, hi, S = slab(N, world, r)
        S0 = S if S0 is None else S0
        assert S == S0 and S % 64 == 0 and S >= 64
        assert 0 <= lo <= hi <= N and hi - lo <= S
        assert lo == min(N, r * S)
        covered.extend(range(lo, hi)) if N < 10000 else covered.append((lo, hi))
    if N < 10000:
        assert covered == list(range(N))
    else:
        assert covered[0][0] == 0 and covered[-1][1] == N
        assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


def test_slab_rejects_bad_args(L):
    from mdqtplasmasims_amd.engine import slab
    from mdqtplasmasims_amd import MdqtError
    with pytest.raises(MdqtError):
        slab(10, 2, 2)
    with pytest.raises(MdqtError):
        slab(10, 0, 0)


def test_create_fails_loudly_without_gpu(L):
    from mdqtplasmasims_amd import MdqtError, Simulation, device_count
    if device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(MdqtError, match="no HIP device"):
        Simulation(N0=100)


def test_bad_rng_configurations_are_rejected(L):
    from mdqtplasmasims_amd import MdqtError, Simulation
    with pytest.raises(MdqtError, match="rng_mode must be"):
        Simulation(N0=100, rng_mode=5)
    # one sequential drand48 stream cannot be sharded
    with pytest.raises(MdqtError, match="needs world_size 1"):
        Simulation(N0=100, rng_mode=0, world_size=2, rank=0)


def test_cli_usage(L):
    import subprocess
    from mdqtplasmasims_amd import CLI_PATH
    r = subprocess.run([CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 2 and "usage: mdqt <job>" in r.stderr
    r = subprocess.run([CLI_PATH, "1", "--bogus=3"], capture_output=True, text=True)
    assert r.returncode == 2


def test_no_oracle_in_product_path():
    """The product package never imports, links or executes the oracle."""
    pkg = os.path.join(ROOT, "mdqtplasmasims_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h", "Makefile")):
                txt = open(os.path.join(dp, f), errors="replace").read()
                for pat in (r"\bimport\s+oracle", r"from\s+oracle", r"liboracle", r"\borc_\w+\(",
                            r"mdqt_oracle", r"oracle/", r"libmdref"):
                    assert not re.search(pat, txt), (f, pat)


# ---- include/mdmc.h (the Monte-Carlo + MD analytics program) ----
MDMC_HEADER = os.path.join(ROOT, "include", "mdmc.h")


def mdmc_header_symbols():
    src = re.sub(r"/\*.*?\*/", "", open(MDMC_HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(mdmc_[A-Za-z0-9_]+)\s*\(", src)))


def test_mdmc_library_exports_and_binding_cover_header(L):
    from mdqtplasmasims_amd._lib import MDMC_SIGNATURES
    syms = mdmc_header_symbols()
    assert {"mdmc_init", "mdmc_monte_carlo", "mdmc_md_steps", "mdmc_pair_corr", "mdmc_autocorrelations",
            "mdmc_tag_particles", "mdmc_tagged_moments", "mdmc_run"} <= set(syms)
    assert not [s for s in syms if not hasattr(L, s)]
    assert set(syms) == {s[0] for s in MDMC_SIGNATURES}


def test_mdmc_params_layout_and_reference_defaults(L):
    from mdqtplasmasims_amd._lib import MdmcParams
    from mdqtplasmasims_amd.mdmc import default_params
    src = open(MDMC_HEADER).read()
    body = src[src.index("typedef struct mdmc_params {"):src.index("} mdmc_params;")]
    names = re.findall(r"\b(?:double|int|uint32_t|char)\s+(\w+)", body)
    assert names == [f[0] for f in MdmcParams._fields_]
    p = default_params()
    # MCMD:62-107
    assert (p.N, p.kappa, p.Gamma, p.n, p.collisionFreq) == (4096, 0.5, 3, 0.4, 0.25)
    assert (p.monteCarloSteps, p.maxRStep, p.pairPairStep, p.timeStep) == (200000, 0.3, 0.05, 0.005)
    assert (p.numPreRecordMDSteps, p.numVelAutoCorrsSteps, p.numInstantaneousAnisotropySteps,
            p.numReestablishEquilSteps) == (200, 2500, 2500, 500)
    assert (p.tempPercentDiff, p.applyForceAlongOneAxisOnly, p.beta, p.anisotropyEstablishmentTime,
            p.anisotropyFromForcesRelaxSteps) == (0.15, 0, 26000, 10, 2000)
    assert p.saveDirectory == b"data/"


def test_mdmc_cli_usage(L):
    import subprocess
    from mdqtplasmasims_amd._lib import MDMC_CLI_PATH
    r = subprocess.run([MDMC_CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 2 and "usage: mdmc <job>" in r.stderr
    r = subprocess.run([MDMC_CLI_PATH, "1", "--bogus=3"], capture_output=True, text=True)
    assert r.returncode == 2
