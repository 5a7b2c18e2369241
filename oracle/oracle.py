"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of the plain-C restatement of the reference hot path (oracle/mdqt_oracle.c) and of
the reference's own MD-only program built unmodified (oracle/_ref/libmdref.so, see
oracle/ref/Makefile).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product package (mdqtplasmasims_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libmdref.so")

_dp = C.POINTER(C.c_double)


class OrcParams(C.Structure):
    _fields_ = [
        ("Ge", C.c_double), ("tmax", C.c_double), ("density", C.c_double), ("sig0", C.c_double),
        ("Te", C.c_double), ("fracOfSig", C.c_double), ("detuning", C.c_double),
        ("detuningDP", C.c_double), ("Om", C.c_double), ("OmDP", C.c_double),
        ("N0", C.c_int), ("newRun", C.c_int), ("c0", C.c_int), ("sampleFreq", C.c_int),
        ("reNormalizewvFns", C.c_int), ("qt_enabled", C.c_int), ("rng_mode", C.c_int),
        ("seed", C.c_uint32), ("job", C.c_uint32), ("nthreads", C.c_int), ("qt_model", C.c_int),
        ("saveDirectory", C.c_char * 256),
        ("tpumpreal", C.c_double), ("tstartV0", C.c_double),
    ]


def build(quiet: bool = True) -> None:
    """Compile the oracle (and, when /root/reference is present, the reference MD build)."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.run(["make", "-C", HERE], check=True, stdout=out)
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-C", os.path.join(HERE, "ref")], check=True, stdout=out)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_default_params.argtypes = [C.POINTER(OrcParams)]
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(OrcParams)]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_get_const.restype = C.c_double
        L.orc_get_const.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_init.argtypes = [C.c_void_p]
        L.orc_get_N.argtypes = [C.c_void_p]
        L.orc_set_state.argtypes = [C.c_void_p, C.c_int, _dp, _dp, C.c_size_t, _dp, _dp, C.c_double]
        L.orc_get_state.argtypes = [C.c_void_p, _dp, _dp, _dp, C.c_size_t, _dp, _dp, _dp]
        L.orc_set_forces.argtypes = [C.c_void_p, _dp, C.c_size_t]
        L.orc_get_time.restype = C.c_double
        L.orc_get_time.argtypes = [C.c_void_p]
        L.orc_set_time.argtypes = [C.c_void_p, C.c_double]
        L.orc_get_qstep_index.restype = C.c_uint64
        L.orc_get_qstep_index.argtypes = [C.c_void_p]
        L.orc_set_qstep_index.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_set_drand48_state.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_get_drand48_state.restype = C.c_uint64
        L.orc_get_drand48_state.argtypes = [C.c_void_p]
        L.orc_get_counters.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint),
                                       _dp, _dp]
        L.orc_forces.argtypes = [C.c_void_p]
        L.orc_forces_raw.argtypes = [C.c_int, C.c_double, C.c_double, _dp, C.c_size_t, _dp, C.c_int]
        L.orc_forces_rows.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, _dp,
                                      C.c_size_t, _dp, C.c_int]
        L.orc_forces_index.argtypes = [C.c_int, C.c_double, C.c_double, _dp, C.c_size_t,
                                       C.POINTER(C.c_int), C.c_int, _dp, C.c_int]
        L.orc_potentials_index.argtypes = [C.c_int, C.c_double, C.c_double, _dp, C.c_size_t,
                                           C.POINTER(C.c_int), C.c_int, _dp, C.c_int]
        L.orc_set_ion_ids.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
        L.orc_epotential.restype = C.c_double
        L.orc_epotential.argtypes = [C.c_void_p]
        L.orc_epotential_raw.restype = C.c_double
        L.orc_epotential_raw.argtypes = [C.c_int, C.c_double, C.c_double, _dp, C.c_size_t]
        L.orc_step.argtypes = [C.c_void_p]
        L.orc_qstep.argtypes = [C.c_void_p]
        L.orc_substeps.argtypes = [C.c_void_p, C.c_int]
        L.orc_md_steps.argtypes = [C.c_void_p, C.c_int]
        L.orc_observables.argtypes = [C.c_void_p, _dp, _dp, _dp]
        L.orc_run.argtypes = [C.c_void_p]
        L.orc_output.argtypes = [C.c_void_p]
        L.orc_write_conditions.argtypes = [C.c_void_p, C.c_int]
        L.orc_read_conditions.argtypes = [C.c_void_p, C.c_int]
        L.orc_setup_directories.argtypes = [C.c_void_p]
        L.orc_save_directory.restype = C.c_char_p
        L.orc_save_directory.argtypes = [C.c_void_p]
        L.orc_drand48_next.restype = C.c_double
        L.orc_drand48_next.argtypes = [C.POINTER(C.c_uint64)]
        L.orc_srand48_state.restype = C.c_uint64
        L.orc_srand48_state.argtypes = [C.c_uint32]
        L.orc_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]
        L.orc_philox_uniform.restype = C.c_double
        L.orc_philox_uniform.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_int]
        L.orc_qstep_ion.argtypes = [C.c_void_p, C.c_double, _dp, _dp, _dp, _dp, C.POINTER(C.c_int)]
        L.orc_tag_spin_up.restype = C.c_int
        L.orc_set_qt_constants.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_double, C.c_double]
        L.orc_tag_spin_up.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        L.orc_run_pump.argtypes = [C.c_void_p]
        L.orc_get_spin_up_list.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def default_params(**kw) -> OrcParams:
    p = OrcParams()
    lib().orc_default_params(C.byref(p))
    for k, v in kw.items():
        if k == "saveDirectory":
            p.saveDirectory = v.encode() if isinstance(v, str) else v
        else:
            setattr(p, k, v)
    return p


class OracleSim:
    """Owning wrapper of one orc_sim (state arrays are copied in / out as numpy)."""

    def __init__(self, **params):
        self.params = default_params(**params)
        self.h = lib().orc_create(C.byref(self.params))
        if not self.h:
            raise MemoryError("orc_create failed")

    def close(self):
        if self.h:
            lib().orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def const(self, name: str) -> float:
        return lib().orc_get_const(self.h, name.encode())

    def init(self):
        if lib().orc_init(self.h) != 0:
            raise RuntimeError("orc_init failed")
        return self

    @property
    def N(self) -> int:
        return lib().orc_get_N(self.h)

    @property
    def t(self) -> float:
        return lib().orc_get_time(self.h)

    @t.setter
    def t(self, v: float):
        lib().orc_set_time(self.h, v)

    @property
    def qstep_index(self) -> int:
        return lib().orc_get_qstep_index(self.h)

    @qstep_index.setter
    def qstep_index(self, q: int):
        lib().orc_set_qstep_index(self.h, q)

    def counters(self):
        c0 = C.c_int(); cnt = C.c_uint(); e = C.c_double(); e0 = C.c_double()
        lib().orc_get_counters(self.h, C.byref(c0), C.byref(cnt), C.byref(e), C.byref(e0))
        return dict(c0=c0.value, counter=cnt.value, Epot=e.value, Epot0=e0.value)

    def get_state(self):
        N = self.N
        R = np.zeros((3, N)); V = np.zeros((3, N)); F = np.zeros((3, N))
        psi = np.zeros((N, 12, 2)); tp = np.zeros(N); t = C.c_double()
        lib().orc_get_state(self.h, _p(R), _p(V), _p(F), N, _p(psi), _p(tp), C.byref(t))
        return dict(R=R, V=V, F=F, psi=psi, tPart=tp, t=t.value)

    def set_state(self, R, V, psi, tPart, t):
        R = np.ascontiguousarray(R, dtype=np.float64); V = np.ascontiguousarray(V, dtype=np.float64)
        psi = np.ascontiguousarray(psi, dtype=np.float64)
        tPart = np.ascontiguousarray(tPart, dtype=np.float64)
        N = R.shape[1]
        lib().orc_set_state(self.h, N, _p(R), _p(V), N, _p(psi), _p(tPart), float(t))

    def set_forces(self, F):
        F = np.ascontiguousarray(F, dtype=np.float64)
        lib().orc_set_forces(self.h, _p(F), F.shape[1])

    def forces(self):
        lib().orc_forces(self.h)

    def epotential(self) -> float:
        return lib().orc_epotential(self.h)

    def step(self):
        lib().orc_step(self.h)

    def qstep(self):
        lib().orc_qstep(self.h)

    def tag_spin_up(self):
        """measureSpinUps / tagParticles of the pumping models: (tags[N], n_up)"""
        tags = np.zeros(self.N, dtype=np.int32)
        n = lib().orc_tag_spin_up(self.h, tags.ctypes.data_as(C.POINTER(C.c_int)))
        return tags, n

    def substeps(self, n: int):
        lib().orc_substeps(self.h, n)

    def md_steps(self, n: int):
        lib().orc_md_steps(self.h, n)

    def observables(self, kde: bool = True, pops: bool = True):
        o = np.zeros(7)
        P = np.zeros((3, 2001)) if kde else None
        pp = np.zeros((self.N, 3)) if pops else None
        lib().orc_observables(self.h, _p(o), _p(P) if kde else None, _p(pp) if pops else None)
        return o, P, pp

    def run(self):
        return lib().orc_run(self.h)

    def run_pump(self):
        """the optical-pumping programs' main() (randomFrozenStartTag408Linear.cpp:981-1076)"""
        return lib().orc_run_pump(self.h)

    def spin_up_list(self):
        tags = np.zeros(self.N, dtype=np.int32)
        n = lib().orc_get_spin_up_list(self.h, tags.ctypes.data_as(C.POINTER(C.c_int)))
        return tags, n

    def output(self):
        return lib().orc_output(self.h)

    def write_conditions(self, c0: int):
        return lib().orc_write_conditions(self.h, c0)

    def read_conditions(self, c0: int):
        return lib().orc_read_conditions(self.h, c0)

    def setup_directories(self):
        return lib().orc_setup_directories(self.h)

    @property
    def save_directory(self) -> str:
        return lib().orc_save_directory(self.h).decode()

    def set_qt_constants(self, dtQ, gamToE, pv2q, r):
        lib().orc_set_qt_constants(self.h, dtQ, gamToE, pv2q, r)

    def set_ion_ids(self, ids):
        """Philox ion key of local ion i = ids[i]: a sampled subset of a larger system draws the
        uniforms its ions draw in the full system"""
        self._ids = np.ascontiguousarray(ids, dtype=np.uint64)
        lib().orc_set_ion_ids(self.h, self._ids.ctypes.data_as(C.POINTER(C.c_uint64)), len(self._ids))

    def qstep_ion(self, t, psi, vx, tPart, u):
        psi = np.ascontiguousarray(psi, dtype=np.float64).copy()
        vxc = C.c_double(vx); tp = C.c_double(tPart)
        uu = np.ascontiguousarray(u, dtype=np.float64)
        nd = C.c_int()
        j = lib().orc_qstep_ion(self.h, t, _p(psi), C.byref(vxc), C.byref(tp), _p(uu), C.byref(nd))
        return dict(jumped=bool(j), psi=psi, vx=vxc.value, tPart=tp.value, ndraws=nd.value)


def forces_raw(R, L, lDeb, nthreads=1):
    R = np.ascontiguousarray(R, dtype=np.float64)
    N = R.shape[1]
    F = np.zeros((3, N))
    lib().orc_forces_raw(N, L, lDeb, _p(R), N, _p(F), nthreads)
    return F


def forces_rows(R, lo, hi, L, lDeb, nthreads=1):
    R = np.ascontiguousarray(R, dtype=np.float64)
    N = R.shape[1]
    F = np.zeros((3, N))
    lib().orc_forces_rows(N, lo, hi, L, lDeb, _p(R), N, _p(F), nthreads)
    return F


def forces_index(R, idx, L, lDeb, nthreads=1):
    """F[3][len(idx)] of the ions idx over all j (SpeedUp:192-236), for sampled-row checks"""
    R = np.ascontiguousarray(R, dtype=np.float64)
    N = R.shape[1]
    ii = np.ascontiguousarray(idx, dtype=np.int32)
    F = np.zeros((3, len(ii)))
    lib().orc_forces_index(N, L, lDeb, _p(R), N, ii.ctypes.data_as(C.POINTER(C.c_int)), len(ii), _p(F), nthreads)
    return F


def potentials_index(R, idx, L, lDeb, nthreads=1):
    """U[len(idx)]: the pair-potential row sums (SpeedUp:256-266's terms) of the ions idx over all j,
    compensated, for sampled-row checks of Epotential() at large N"""
    R = np.ascontiguousarray(R, dtype=np.float64)
    N = R.shape[1]
    ii = np.ascontiguousarray(idx, dtype=np.int32)
    U = np.zeros(len(ii))
    lib().orc_potentials_index(N, L, lDeb, _p(R), N, ii.ctypes.data_as(C.POINTER(C.c_int)), len(ii), _p(U), nthreads)
    return U


def epotential_raw(R, L, lDeb):
    R = np.ascontiguousarray(R, dtype=np.float64)
    return lib().orc_epotential_raw(R.shape[1], L, lDeb, _p(R), R.shape[1])


def philox4x32_10(ctr, key):
    c = (C.c_uint32 * 4)(*ctr); k = (C.c_uint32 * 2)(*key); o = (C.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def philox_uniform(seed, job, ion, qstep, draw):
    return lib().orc_philox_uniform(seed, job, ion, qstep, draw)


def drand48_stream(seed: int, n: int):
    x = C.c_uint64(lib().orc_srand48_state(seed))
    return np.array([lib().orc_drand48_next(C.byref(x)) for _ in range(n)])


# ---------------------------------------------------------------------------------------------
# the reference's own compiled MD code (oracle/_ref/libmdref.so)
# ---------------------------------------------------------------------------------------------
_ref = None


def ref_available() -> bool:
    return os.path.exists(REF_LIB_PATH)


def ref():
    global _ref
    if _ref is None:
        L = C.CDLL(REF_LIB_PATH)
        for n in ("mdref_L", "mdref_rcut", "mdref_kappa"):
            getattr(L, n).restype = C.c_double
        L.mdref_uij.restype = C.c_double
        L.mdref_uij.argtypes = [C.c_double]
        L.mdref_aij.restype = C.c_double
        L.mdref_aij.argtypes = [C.c_double]
        L.mdref_accelerations.argtypes = [_dp, _dp]
        L.mdref_particle_potentials.argtypes = [_dp, _dp]
        L.mdref_step_positions.argtypes = [_dp, _dp, _dp]
        _ref = L
    return _ref


def ref_accelerations(R):
    R = np.ascontiguousarray(R, dtype=np.float64)
    assert R.shape == (3, 4096)
    A = np.zeros((3, 4096))
    ref().mdref_accelerations(_p(R), _p(A))
    return A


def ref_particle_potentials(R):
    R = np.ascontiguousarray(R, dtype=np.float64)
    U = np.zeros(4096)
    ref().mdref_particle_potentials(_p(R), _p(U))
    return U


def ref_step_positions(R, V, A):
    R = np.ascontiguousarray(R, dtype=np.float64).copy()
    V = np.ascontiguousarray(V, dtype=np.float64); A = np.ascontiguousarray(A, dtype=np.float64)
    ref().mdref_step_positions(_p(R), _p(V), _p(A))
    return R


class RefMCMD:
    """The reference's MonteCarloFollowedByMDAndTempAnisotropy.cpp program state (its globals in
    oracle/_ref/libmdref.so, one instance per process), with its mt19937 reseeded.  Stages are the
    reference's own functions (oracle/ref/ref_harness.cpp)."""

    N = 4096
    T = 2500

    def __init__(self, seed: int, save_directory: str = "data/"):
        L = ref()
        if not getattr(L, "_mcmd_bound", False):
            L.mdref_seed.argtypes = [C.c_uint]
            L.mdref_set_collision_freq.argtypes = [C.c_double]
            L.mdref_set_laser_force.argtypes = [C.c_int]
            L.mdref_set_save_directory.argtypes = [C.c_char_p]
            L.mdref_get.argtypes = [_dp, _dp, _dp, _dp]
            L.mdref_set.argtypes = [_dp, _dp, _dp, _dp]
            L.mdref_monte_carlo.argtypes = [C.c_int]
            L.mdref_md_steps.argtypes = [C.c_int]
            L.mdref_pair_corr.argtypes = [C.c_int]
            L.mdref_autocorrelations.argtypes = [_dp, C.c_int, _dp]
            L.mdref_record_temp_axes.argtypes = [C.c_int]
            L.mdref_tag_particles.argtypes = [C.POINTER(C.c_int)]
            L.mdref_tagged_moments.argtypes = [C.c_int]
            L._mcmd_bound = True
        self.L = L
        L.mdref_seed(int(seed))
        L.mdref_set_collision_freq(0.25)
        L.mdref_set_laser_force(0)
        self.set_save_directory(save_directory)

    def set_save_directory(self, d: str):
        self.L.mdref_set_save_directory(d.encode())

    def init(self):
        self.L.mdref_init()

    def monte_carlo(self, n: int):
        self.L.mdref_monte_carlo(int(n))

    def md_steps(self, n: int):
        self.L.mdref_md_steps(int(n))

    def set_collision_freq(self, f: float):
        self.L.mdref_set_collision_freq(float(f))

    def set_laser_force(self, on: bool):
        self.L.mdref_set_laser_force(int(bool(on)))

    def get_state(self):
        R = np.zeros((3, 4096)); V = np.zeros((3, 4096)); A = np.zeros((3, 4096)); U = np.zeros(4096)
        self.L.mdref_get(_p(R), _p(V), _p(A), _p(U))
        return R, V, A, U

    def set_state(self, R=None, V=None, A=None, U=None):
        arr = [None if x is None else np.ascontiguousarray(x, dtype=np.float64) for x in (R, V, A, U)]
        self.L.mdref_set(*[None if x is None else _p(x) for x in arr])

    def pair_corr_file(self, step: int):      # writes <dir>pairPairCorrStepNum<step>.dat
        self.L.mdref_pair_corr(int(step))

    def autocorrelations(self, vs: np.ndarray) -> np.ndarray:   # vs [3][4096][T] -> [4][T]
        vs = np.ascontiguousarray(vs, dtype=np.float64)
        T = vs.shape[2]
        out = np.zeros((4, 2500))
        self.L.mdref_autocorrelations(_p(vs), T, _p(out))
        return out[:, :T]

    def record_temperature(self):
        self.L.mdref_record_temperature()

    def record_temp_axes(self, step: int):
        self.L.mdref_record_temp_axes(int(step))

    def tag_particles(self) -> np.ndarray:
        t = np.zeros((4, 4096), dtype=np.int32)
        self.L.mdref_tag_particles(t.ctypes.data_as(C.POINTER(C.c_int)))
        return t

    def tagged_moments_file(self, step: int):
        self.L.mdref_tagged_moments(int(step))


# ---------------------------------------------------------------------------------------------
# restatements for MonteCarloFollowedByMDAndTempAnisotropy.cpp ("MCMD")
# ---------------------------------------------------------------------------------------------
def mcmd_autocorrelations(vs: np.ndarray, Gamma: float) -> np.ndarray:
    """VAF, longViscAutoCorr, vCubeAutoCorr, vFourthAutoCorr of MCMD:655-807 over vs [3][N][T]:
    out[f][td] = sum_{i, j < T-td} term_f(j, j+td) / (N (T - td)), with the -3/Gamma^2 and
    -27/Gamma^4 offsets of :710 / :785 applied once per term.  Lag sums through a zero-padded
    FFT (float64): equal to the reference's direct sums up to summation rounding."""
    vs = np.asarray(vs, dtype=np.float64)
    _, N, T = vs.shape
    n = 1 << int(np.ceil(np.log2(2 * T)))

    def lagsum(a):                      # sum over (component, particle) of sum_j a[j] a[j + td]
        f = np.fft.rfft(a, n=n, axis=-1)
        return np.fft.irfft((f * np.conj(f)).sum(axis=(0, 1)), n=n)[:T]

    cnt = N * (T - np.arange(T)).astype(np.float64)
    v2 = vs * vs
    out = np.empty((4, T))
    out[0] = lagsum(vs) / cnt
    out[1] = lagsum(v2) / cnt - 3 / (Gamma * Gamma)
    out[2] = lagsum(v2 * vs) / cnt
    out[3] = lagsum(v2 * v2) / cnt - 3 * 9 / (Gamma * Gamma * Gamma * Gamma)
    return out


class MT19937:
    """std::mt19937 (C++ [rand.predef]) + libstdc++'s generate_canonical<double, 53> behind
    uniform_real_distribution<double>(0, 1) (MCMD:53-54): u = (g1 + g2 2^32) / 2^64, values >= 1
    mapped to the largest double below 1.  The restatement the device MC kernel follows."""

    def __init__(self, seed: int = 5489):
        x = [0] * 624
        x[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            x[i] = (1812433253 * (x[i - 1] ^ (x[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.x, self.p = x, 624

    def _twist(self):
        x = self.x
        for k in range(624):
            y = (x[k] & 0x80000000) | (x[(k + 1) % 624] & 0x7FFFFFFF)
            x[k] = x[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.p = 0

    def __call__(self) -> int:
        if self.p >= 624:
            self._twist()
        z = self.x[self.p]
        self.p += 1
        z ^= z >> 11
        z ^= (z << 7) & 0x9D2C5680
        z ^= (z << 15) & 0xEFC60000
        z ^= z >> 18
        return z & 0xFFFFFFFF

    def uniform(self) -> float:
        s = float(self())
        s = s + float(self()) * 4294967296.0
        r = s / 18446744073709551616.0
        return r if r < 1.0 else float(np.nextafter(1.0, 0.0))
