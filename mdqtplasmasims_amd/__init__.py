"""mdqtplasmasims_amd — MI355X-native engine for the Yukawa-OCP MD + per-ion quantum-trajectory
(MDQT) hot path of tlangin/MDQTPlasmaSims' laserCoolingPlusExpansionMDQTSpeedUp.cpp.

Native code: mdqtplasmasims_amd/csrc (HIP kernels for gfx950 + C++ host engine) built into
mdqtplasmasims_amd/lib/libmdqt.so with the C ABI of include/mdqt.h.  This package is the Python
mirror of the reference's function seam (engine.Simulation) and the multi-GPU driver (sharded).
"""
from ._lib import MdqtError, LIB_PATH, CLI_PATH  # noqa: F401
from .engine import Simulation, default_params, device_count, slab  # noqa: F401

__all__ = ["Simulation", "MdqtError", "default_params", "device_count", "slab", "LIB_PATH", "CLI_PATH"]
