"""the CPU restatement's OpenMP loops under ThreadSanitizer (clang -fsanitize=thread,
LLVM libomp + libarcher so that TSan sees OpenMP's barriers).  The oracle run must be clean; the
positive control — the reference's Newton-3 scatter pattern in an OpenMP loop (SpeedUp:228-230) —
must be reported, which shows the sanitizer sees races in this setup.  No GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/llvm"
ARCHER = os.path.join(LLVM, "lib", "libarcher.so")
EXE = os.path.join(ROOT, "oracle", "_tsan", "tsan_harness")


@pytest.fixture(scope="module")
def harness():
    if not (os.path.exists(os.path.join(LLVM, "bin", "clang")) and os.path.exists(ARCHER)):
        pytest.skip("clang / libarcher not available")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle", "tsan")], check=True)
    return EXE


def run(exe, mode):
    env = dict(os.environ, OMP_TOOL_LIBRARIES=ARCHER, TSAN_OPTIONS="halt_on_error=0 exitcode=0 ignore_noninstrumented_modules=1")
    r = subprocess.run([exe, mode], env=env, capture_output=True, text=True, timeout=300)
    return r.returncode, r.stdout + r.stderr


def test_oracle_openmp_loops_are_race_free(harness):
    rc, out = run(harness, "oracle")
    assert rc == 0, out[-2000:]
    assert "oracle N=" in out
    assert "ThreadSanitizer" not in out.replace("Archer detected OpenMP application with TSan", ""), out[-3000:]


def test_tsan_reports_the_reference_scatter_race(harness):
    rc, out = run(harness, "control")
    assert "WARNING: ThreadSanitizer: data race" in out, out[-2000:]
