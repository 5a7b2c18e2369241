"""Python mirror of MonteCarloFollowedByMDAndTempAnisotropy.cpp ("MCMD", tlangin/MDQTPlasmaSims):
Metropolis anneal of a Yukawa OCP, velocity-Verlet MD with collisions and an anisotropic laser
force, and the program's analytics (g(r), velocity autocorrelations, tagged-particle moments,
temperatures).  Every method calls the C ABI of include/mdmc.h (libmdqt.so, gfx950 kernels);
there is no CPU fallback.  Method names follow the reference's functions.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MdmcParams, check, dptr, lib


def default_params(**over) -> MdmcParams:
    """MCMD:62-107 defaults, with keyword overrides."""
    p = MdmcParams()
    lib().mdmc_default_params(C.byref(p))
    for k, v in over.items():
        if k == "saveDirectory":
            v = v.encode() if isinstance(v, str) else v
        if not hasattr(p, k):
            raise AttributeError(f"mdmc_params has no field {k}")
        setattr(p, k, v)
    return p


class MonteCarloMD:
    """One MCMD system resident on a GPU (R, V, A, U and the velocity store in HBM)."""

    def __init__(self, params: MdmcParams | None = None, **over):
        self.p = params if params is not None else default_params(**over)
        h = C.c_void_p()
        check(lib().mdmc_create(C.byref(self.p), C.byref(h)), "mdmc_create")
        self._h = h
        self.N = int(self.p.N)
        self.T = int(self.p.numVelAutoCorrsSteps)

    def close(self):
        if getattr(self, "_h", None):
            lib().mdmc_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def const(self, name: str) -> float:
        return lib().mdmc_get_const(self._h, name.encode())

    # ---- the program's functions ----
    def init(self):                                   # init() :173-203 + potentials :207-245
        check(lib().mdmc_init(self._h), "mdmc_init")

    def monte_carlo(self, nsteps: int) -> int:       # MonteCarloStep() x n :315-382
        acc = C.c_longlong(0)
        check(lib().mdmc_monte_carlo(self._h, int(nsteps), C.byref(acc)), "mdmc_monte_carlo")
        return int(acc.value)

    def md_steps(self, nsteps: int):                 # MDStep() x n :504-511
        check(lib().mdmc_md_steps(self._h, int(nsteps)), "mdmc_md_steps")

    def set_collision_freq(self, f: float):
        check(lib().mdmc_set_collision_freq(self._h, float(f)))

    def set_laser_force(self, on: bool):
        check(lib().mdmc_set_laser_force(self._h, int(bool(on))))

    def pair_corr(self) -> np.ndarray:               # recordPairPairCorr :584-652
        nb = C.c_int(0)
        check(lib().mdmc_pair_corr(self._h, None, 0, C.byref(nb)), "mdmc_pair_corr")
        g = np.zeros(nb.value)
        check(lib().mdmc_pair_corr(self._h, dptr(g), g.size, C.byref(nb)), "mdmc_pair_corr")
        return g

    def record_velocities(self, k: int):             # recordVelsForAutocorrelations :513-523
        check(lib().mdmc_record_velocities(self._h, int(k)), "mdmc_record_velocities")

    def set_velocity_store(self, vs: np.ndarray):    # [3][N][T]
        vs = np.ascontiguousarray(vs, dtype=np.float64)
        if vs.shape != (3, self.N, self.T):
            raise ValueError(f"velocity store must be (3, {self.N}, {self.T})")
        check(lib().mdmc_set_velocity_store(self._h, dptr(vs)), "mdmc_set_velocity_store")

    def autocorrelations(self) -> np.ndarray:        # VAF, longVisc, vCube, vFourth :655-807
        out = np.zeros((4, self.T))
        check(lib().mdmc_autocorrelations(self._h, dptr(out)), "mdmc_autocorrelations")
        return out

    def temperatures(self) -> np.ndarray:            # recordTemperature, recordTempForEachAxis
        out = np.zeros(4)
        check(lib().mdmc_temperatures(self._h, dptr(out)), "mdmc_temperatures")
        return out

    def anisotropize(self):                          # anisotropizeVelocities :548-558
        check(lib().mdmc_anisotropize(self._h), "mdmc_anisotropize")

    def tag_particles(self) -> np.ndarray:           # tagParticles :810-921 -> [4][N] 0/1
        t = np.zeros((4, self.N), dtype=np.int32)
        check(lib().mdmc_tag_particles(self._h, t.ctypes.data_as(C.POINTER(C.c_int))), "mdmc_tag_particles")
        return t

    def tagged_moments(self) -> np.ndarray:          # recordTaggedParticleMoments :923-1028 -> [4][4]
        out = np.zeros(16)
        check(lib().mdmc_tagged_moments(self._h, dptr(out)), "mdmc_tagged_moments")
        return out.reshape(4, 4)

    def get_state(self):
        R = np.zeros((3, self.N)); V = np.zeros((3, self.N)); A = np.zeros((3, self.N)); U = np.zeros(self.N)
        check(lib().mdmc_get_state(self._h, dptr(R), dptr(V), dptr(A), dptr(U)), "mdmc_get_state")
        return R, V, A, U

    def set_state(self, R=None, V=None, A=None, U=None):
        arr = [None if x is None else np.ascontiguousarray(x, dtype=np.float64) for x in (R, V, A, U)]
        check(lib().mdmc_set_state(self._h, *[dptr(x) for x in arr]), "mdmc_set_state")

    def setup_directories(self) -> str:              # main() :1037-1058
        check(lib().mdmc_setup_directories(self._h), "mdmc_setup_directories")
        return lib().mdmc_save_directory(self._h).decode()

    def run(self, verbose: bool = False):            # main() :1030-1167
        check(lib().mdmc_run(self._h, int(bool(verbose))), "mdmc_run")
