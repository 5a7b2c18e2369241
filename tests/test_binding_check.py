"""The reference-side binding of INTEGRATION.md, compiled and driven.

tests/native/binding_check.cpp keeps SpeedUp's shape — its globals, `void f(void)` functions and
main()'s time loop (laserCoolingPlusExpansionMDQTSpeedUp.cpp:1139-1383) — with the INTEGRATION.md
stubs as the function bodies: forces(), step() and qstep() one call each per substep, output(),
writeConditions(), Epotential(), init() = the reference's host drand48 sampling + push_state(),
readConditions() = mdqt_read_conditions + pull_state().  Built by __graft_entry__.build() (g++,
linked to mdqtplasmasims_amd/lib/libmdqt.so).

The GPU test runs it and mdqt_run (the engine's own main loop: fused substeps, device init()) with
the same inputs and requires the two output trees to be identical file for file, byte for byte —
energies.dat, the vel_dist / statePopulations files of every output(), ions_ / conditions_ / VZERO_ /
wvFns_ of writeConditions — then resumes both from their own files (newRun 0, readConditions(c0))
and compares again."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "binding_check")


def _tree(base):
    out = {}
    for d, _, fs in os.walk(base):
        for f in fs:
            p = os.path.join(d, f)
            with open(p, "rb") as fh:
                out[os.path.relpath(p, base)] = fh.read()
    return out


def test_binding_check_source_binds_every_stub():
    """CPU: the check program binds exactly the INTEGRATION.md stubs (and is built by build())"""
    src = open(os.path.join(ROOT, "tests", "native", "binding_check.cpp")).read()
    for fn, call in (("forces", "mdqt_forces"), ("step", "mdqt_step"), ("qstep", "mdqt_qstep"),
                     ("Epotential", "mdqt_epotential"), ("output", "mdqt_output"),
                     ("writeConditions", "mdqt_write_conditions"), ("readConditions", "mdqt_read_conditions")):
        assert re.search(r"void %s\([^)]*\) \{ mdqt_or_die\(%s\(" % (fn, call), src), fn
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for name in ("mdqt_attach", "push_state", "push_counters", "pull_state", "void init(void)", "readConditions"):
        assert name in integ, name
    assert "binding_check" in open(os.path.join(ROOT, "__graft_entry__.py")).read()


@pytest.mark.gpu
def test_reference_binding_files_identical_to_mdqt_run(tmp_path):
    import mdqtplasmasims_amd as M
    assert os.path.exists(EXE), "tests/native/binding_check missing: run __graft_entry__.build()"
    N0, tmax, sf, seed, job = 500, 0.1, 10, 12346, 1
    a, b = str(tmp_path / "binding") + "/", str(tmp_path / "run") + "/"

    def binding(tm, extra=()):
        r = subprocess.run([EXE, str(job), a, str(N0), str(tm), str(sf), str(seed), *extra],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        m = re.search(r"binding_check: N=(\d+) c0=(-?\d+) t=([0-9.]+)", r.stdout)
        assert m, r.stdout[-500:]
        return int(m.group(1)), int(m.group(2))

    def engine(tm, newRun=1, c0=0):
        s = M.Simulation(N0=N0, tmax=tm, sampleFreq=sf, seed=seed, job=job, saveDirectory=b, newRun=newRun, c0=c0)
        s.run()
        n, c = s.N, s.counters()["c0"]
        s.close()
        return n, c

    na, ca = binding(tmax)
    nb, cb = engine(tmax)
    assert (na, ca) == (nb, cb)
    ta, tb = _tree(a), _tree(b)
    assert sorted(ta) == sorted(tb)
    diff = [k for k in ta if ta[k] != tb[k]]
    print(f"N={na} c0={ca}: {len(ta)} files, {sum(len(v) for v in ta.values())} bytes; differing: {diff[:5]}")
    assert not diff
    assert any(k.endswith("energies.dat") for k in ta) and any("wvFns_timestep" in k for k in ta)
    assert sum(1 for k in ta if "statePopulationsVsVTime" in k) == 5          # output() at c0 = 9, 19, ..., 49
    # resume both from their own files (readConditions(c0), SpeedUp:785-916) for 20 more MD steps
    na2, ca2 = binding(tmax + 0.04, ("0", str(ca)))
    nb2, cb2 = engine(tmax + 0.04, newRun=0, c0=cb)
    assert (na2, ca2) == (nb2, cb2) and ca2 > ca
    ta, tb = _tree(a), _tree(b)
    assert sorted(ta) == sorted(tb)
    diff = [k for k in ta if ta[k] != tb[k]]
    print(f"resumed at c0={ca} to c0={ca2}: {len(ta)} files; differing: {diff[:5]}")
    assert not diff
