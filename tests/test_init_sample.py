"""init()'s rejection sampling (SpeedUp:289-335) run in parallel over one drand48 stream
(mdqtplasmasims_amd/csrc/mdqt_init_sample.hpp) must equal the sequential walk bit for bit: the
kept ions, their wavefunction draws and the stream state the qsteps continue from.  CPU only
(tests/native/init_check.cpp, compiled with g++ here)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "mdqtplasmasims_amd", "csrc")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("init") / "init_check")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-pthread", "-I", CSRC,
                        os.path.join(HERE, "native", "init_check.cpp"), "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.parametrize("N0,seed,threads,nbound,N", [
    (500, 7, 3, 0, None),
    (3500, 12346, 8, 0, 3573),          # C2's realised N
    (3500, 12346, 5, 1000, 3573),       # bound too small: the walk leaves the scanned range, finishes sequentially
    (60, 99, 16, 0, None),
    (30000, 12345, 7, 0, None),
])
def test_parallel_init_equals_sequential(driver, N0, seed, threads, nbound, N):
    r = subprocess.run([driver, str(N0), str(seed), str(threads), str(nbound)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    if N is not None:
        assert r.stdout.startswith(f"N={N} "), r.stdout
