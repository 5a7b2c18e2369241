"""The optical-pumping programs' main() on the GPU (mdqt_run_pump; randomFrozenStartTag408Linear.cpp
:981-1076, 408Quad, 422Linear) against the oracle's restatement of the same flow (orc_run_pump):
directory name, the file set, spinUpIons / spinUpIonsList / ions exactly, energies, taggedMoments,
VAF, vel_distX and conditions to the printed %lg precision (1e-5 relative, a few-ulp difference of
the forces grows over ~150 MD steps), and the resume path (readConditions: spin-up list, the
vel[i] = i 0.0025 bins of :723)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SMALL = dict(N0=300, seed=5, job=2, rng_mode=1, tmax=0.3, sampleFreq=10, tpumpreal=5.2e-8, tstartV0=0.1)


def files(d):
    return sorted(f for f in os.listdir(d))


def numbers(path):
    return np.array([float(x) for x in open(path).read().split()])


def compare_dirs(a, b, tol=1e-5):
    fa, fb = files(a), files(b)
    assert fa == fb, (fa, fb)
    for f in fa:
        ta, tb = open(os.path.join(a, f)).read(), open(os.path.join(b, f)).read()
        if f.startswith(("ions_", "spinUpIons")):
            assert ta == tb, f
            continue
        x, y = numbers(os.path.join(a, f)), numbers(os.path.join(b, f))
        assert x.shape == y.shape, f
        scale = max(np.abs(y).max(), 1e-300)
        assert np.all(np.abs(x - y) <= tol * np.maximum(np.abs(y), 1e-3 * scale)), (f, np.abs(x - y).max())


@pytest.mark.parametrize("model,kw", [(1, dict(Om=0.7, detuning=-2.5)), (2, dict(Om=2.0, detuning=0.0)),
                                      (3, dict(Om=1.3, detuning=-1.0))])
def test_pump_main_matches_oracle(tmp_path, orc, model, kw):
    import mdqtplasmasims_amd as M
    p = dict(SMALL, Ge=0.1, **kw)
    g = M.Simulation(pump_program=model, saveDirectory=str(tmp_path / "gpu") + "/", **p)
    g.run_pump()
    o = orc.OracleSim(qt_model=model, saveDirectory=str(tmp_path / "orc") + "/", **p)
    assert o.run_pump() == 0
    dg, do = g.save_directory, o.save_directory
    assert os.path.basename(os.path.dirname(dg.rstrip("/"))) == os.path.basename(os.path.dirname(do.rstrip("/")))
    assert dg.endswith("/job2/")
    tg, ng = g.spin_up_list()
    to, no = o.spin_up_list()
    assert ng == no and np.array_equal(tg, to) and 0 < ng < g.N
    compare_dirs(dg, do)
    # resume (newRun = 0) from the files just written: readConditions (:709-797), then the loop
    c0 = g.counters()["c0"]
    r = M.Simulation(pump_program=model, saveDirectory=str(tmp_path / "gpu") + "/", newRun=0, c0=c0,
                     **dict(p, tmax=p["tmax"] + 0.05))
    r.run_pump()
    tr, nr = r.spin_up_list()
    assert nr == ng and np.array_equal(tr, tg)
    assert abs(r.t - (p["tmax"] + 0.05)) < 0.01
    idx = max(int(f[len("vel_distX_timestep"):-4]) for f in files(r.save_directory) if f.startswith("vel_distX_"))
    assert idx > c0                                      # written by the resumed run
    dist = os.path.join(r.save_directory, f"vel_distX_timestep{idx:06d}.dat")
    rows = [l.split() for l in open(dist).read().splitlines()]
    assert len(rows) == 4001 and float(rows[0][0]) == 0.0 and abs(float(rows[-1][0]) - 10.0) < 1e-12
    for s in (g, r):
        s.close()
    o.close()


def test_pump_program_directory_names(tmp_path):
    """the directory names of the three programs' default inputs (:990 sprintf with (unsigned) casts)"""
    import mdqtplasmasims_amd as M
    want = {1: "PumpTime200PumpStart15Det250Om70Density20Ge100NumIons3500",
            2: "PumpTime100PumpStart15Det0Om200Density20Ge100NumIons3500",
            3: "PumpTime100PumpStart15Det100Om130Density20Ge100NumIons3500"}
    for model, name in want.items():
        s = M.Simulation(pump_program=model, saveDirectory=str(tmp_path) + "/", N0=3500, tmax=-1.0)
        s.run_pump()                                     # tmax < 0: directories, init(), writeConditions only
        assert os.path.basename(os.path.dirname(s.save_directory.rstrip("/"))) == name, s.save_directory
        s.close()


def test_cli_pump_program(tmp_path):
    """`mdqt <job> --pump_program=3` runs the 422 nm program's main(): its defaults
    (randomFrozenStartTag422Linear.cpp:52-78) overridden by the flags, the PumpTime... tree"""
    import subprocess
    from mdqtplasmasims_amd import CLI_PATH
    r = subprocess.run([CLI_PATH, "2", "--pump_program=3", "--N0=300", "--tmax=0.3", "--sampleFreq=10",
                        "--tpumpreal=5.2e-8", "--tstartV0=0.1", "--seed=5", f"--saveDirectory={tmp_path}/"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    dirs = [d for d in os.listdir(tmp_path) if d.startswith("PumpTime")]
    assert len(dirs) == 1 and dirs[0].endswith("Det100Om130Density20Ge100NumIons300"), dirs
    job = tmp_path / dirs[0] / "job2"
    names = os.listdir(job)
    assert "taggedMoments.dat" in names and "VAF.dat" in names and "energies.dat" in names
    assert any(n.startswith("spinUpIons_timestep") for n in names)
    assert any(n.startswith("vel_distX_timestep") for n in names)
