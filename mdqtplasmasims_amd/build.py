"""Build libmdqt.so and the `mdqt` CLI in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m mdqtplasmasims_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(quiet: bool = False, jobs: int = 4) -> None:
    env = dict(os.environ)
    env.setdefault("HIPCC", "/opt/rocm/bin/hipcc")
    out = subprocess.DEVNULL if quiet else None
    subprocess.run(["make", "-C", os.path.join(HERE, "csrc"), f"-j{jobs}"], check=True, stdout=out, env=env)


if __name__ == "__main__":
    build(quiet="-q" in sys.argv)
