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


def default_params(qt_model: int = 0, **over) -> MdmcParams:
    """MCMD:62-107 defaults (qt_model 1..3: the QT tagging program's, QTT:75-121), with overrides."""
    p = MdmcParams()
    if qt_model:
        check(lib().mdmc_default_params_qt(C.byref(p), int(qt_model)), "mdmc_default_params_qt")
    else:
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

    def run(self, verbose: bool = False):            # main() :1030-1167 (QTT :1140-1254)
        check(lib().mdmc_run(self._h, int(bool(verbose))), "mdmc_run")

    # ---- QT tagging variants (qt_model 1..3) ----
    def qsteps(self, n: int):                        # qstep() x n (QTT:555-756)
        check(lib().mdmc_qsteps(self._h, int(n)), "mdmc_qsteps")

    def tag_qt(self):                                # tagParticles (QTT:1022-1067) -> (tags [N], count)
        t = np.zeros(self.N, dtype=np.int32)
        cnt = C.c_int(0)
        check(lib().mdmc_tag_qt(self._h, t.ctypes.data_as(C.POINTER(C.c_int)), C.byref(cnt)), "mdmc_tag_qt")
        return t, cnt.value

    def tagged_moments_qt(self, dist: bool = True):  # recordTaggedParticleMoments (QTT:1069-1138)
        out = np.zeros(4)
        d = np.zeros((3, 4001)) if dist else None
        check(lib().mdmc_tagged_moments_qt(self._h, dptr(out), dptr(d)), "mdmc_tagged_moments_qt")
        return (out, d) if dist else out

    def get_psi(self) -> np.ndarray:                 # [N][12] complex
        a = np.zeros((self.N, 12, 2))
        check(lib().mdmc_get_psi(self._h, dptr(a)), "mdmc_get_psi")
        return a[..., 0] + 1j * a[..., 1]

    def set_psi(self, psi):
        psi = np.asarray(psi, dtype=complex)
        a = np.ascontiguousarray(np.stack([psi.real, psi.imag], -1), dtype=np.float64)
        check(lib().mdmc_set_psi(self._h, dptr(a)), "mdmc_set_psi")
