"""The output-file writer (mdqtplasmasims_amd/csrc/mdqt_writer.hpp): "%lg" text through
std::to_chars must be byte-identical to the reference's fprintf("%lg") (SpeedUp:725-1032), and the
background writer pool must report I/O errors at its flush.  CPU only: the header is compiled
with g++ into a small driver (tests/native/writer_check.cpp)."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "mdqtplasmasims_amd", "csrc")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("writer")
    exe = str(d / "writer_check")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-I", CSRC,
                        os.path.join(HERE, "native", "writer_check.cpp"), "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def _values(n=240_000, seed=3):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal(n) * 10.0 ** rng.integers(-12, 12, n)
    b = rng.integers(0, 2_000_000, n) / 1e6 * 10.0 ** rng.integers(-6, 6, n)   # rounding boundaries
    c = np.frombuffer(rng.bytes(8 * n), dtype=np.float64).copy()                   # any bit pattern
    special = np.array([0.0, -0.0, 1e-5, 1e-4, 999999.5, 9.999995e-5, 0.5, 5e-324, 1e300,
                        np.inf, -np.inf, np.nan] * 2)
    x = np.concatenate([a, b, np.nextafter(b, np.inf), c, special])
    return x[: len(x) // 24 * 24]


def test_lg_text_is_byte_identical_to_fprintf(driver, tmp_path):
    x = _values()
    x.tofile(tmp_path / "in.bin")
    r = subprocess.run([driver, str(tmp_path / "in.bin"), str(tmp_path)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr)
    for k in range(4):
        a = (tmp_path / f"async{k}.dat").read_bytes()
        b = (tmp_path / f"printf{k}.dat").read_bytes()
        assert a == b, k
    # and the same text as Python's "%g" (correctly rounded, 6 significant digits) for finite rows
    rows = x[: 24 * 50].reshape(-1, 6)[0::4]
    want = "".join("".join("%g\t" % v for v in row) + "\n" for row in rows)
    assert (tmp_path / "async0.dat").read_text()[: len(want)] == want
