"""Python host API of the MI355X MDQT engine — a thin mirror of the reference's function seam.

The reference program (laserCoolingPlusExpansionMDQTSpeedUp.cpp, "SpeedUp") exposes no library:
its hot path is a set of ``void f(void)`` functions over globals (SpeedUp:176-185).  This class keeps
those names and their meaning, over one device-resident simulation held by libmdqt.so:

    ===========================  ==================================  ==========================
    reference (SpeedUp)          here                                C ABI (include/mdqt.h)
    ===========================  ==================================  ==========================
    init()            :289-348   Simulation.init()                   mdqt_init
    forces()          :192-236   Simulation.forces()                 mdqt_forces
    step()            :418-430   Simulation.step()                   mdqt_step
    qstep()           :438-717   Simulation.qstep()                  mdqt_qstep
    step();qstep() x n           Simulation.substeps(n)              mdqt_substeps (fused)
    Epotential()      :244-281   Simulation.Epotential()             mdqt_epotential
    output()          :917-1032  Simulation.output()                 mdqt_output
    writeConditions() :725-784   Simulation.writeConditions(c0)      mdqt_write_conditions
    readConditions()  :785-916   Simulation.readConditions(c0)       mdqt_read_conditions
    main()            :1139-1383 Simulation.run()                    mdqt_run
    ===========================  ==================================  ==========================

Parameters keep the reference's names and defaults (SpeedUp:56-85).  Errors raise MdqtError
(the reference has no error reporting at all: unchecked fopen, void returns).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MdqtError, MdqtParams, check, dptr, lib

NBINS = 2001
NUM_STATES = 12

# reference parameter names (SpeedUp:56-85) plus the engine's extensions
PARAM_NAMES = [f[0] for f in MdqtParams._fields_]


def default_params(**kw) -> MdqtParams:
    p = MdqtParams()
    lib().mdqt_default_params(C.byref(p))
    for k, v in kw.items():
        if k not in PARAM_NAMES:
            raise KeyError(f"unknown parameter {k!r}")
        if k == "saveDirectory":
            p.saveDirectory = v.encode() if isinstance(v, str) else v
        else:
            setattr(p, k, v)
    return p


def default_params_pump(qt_model: int, **kw) -> MdqtParams:
    """the optical-pumping program's defaults (qt_model 1 / 2 / 3 = randomFrozenStartTag408Linear /
    408Quad / 422Linear.cpp globals), then the overrides in kw"""
    p = MdqtParams()
    lib().mdqt_default_params_pump(C.byref(p), int(qt_model))
    for k, v in kw.items():
        if k not in PARAM_NAMES:
            raise KeyError(f"unknown parameter {k!r}")
        if k == "saveDirectory":
            p.saveDirectory = v.encode() if isinstance(v, str) else v
        else:
            setattr(p, k, v)
    return p


def device_count() -> int:
    return lib().mdqt_device_count()


def slab(N: int, world: int, rank: int):
    """(lo, hi, S): ions [lo, hi) owned by `rank`, slab stride S (pure function of N, world)."""
    lo, hi, S = C.c_int(), C.c_int(), C.c_int()
    check(lib().mdqt_slab(N, world, rank, C.byref(lo), C.byref(hi), C.byref(S)), "mdqt_slab")
    return lo.value, hi.value, S.value


def forces_raw(R, L: float, lDeb: float, nseg: int = 0, device: int = -1, variant: int = 1):
    """Yukawa forces of positions R[3][N] in a periodic box L (kernel 1, stateless)."""
    R = np.ascontiguousarray(R, dtype=np.float64)
    N = R.shape[1]
    F = np.zeros((3, N))
    check(lib().mdqt_forces_raw(N, float(L), float(lDeb), dptr(R), N, dptr(F), int(nseg), int(device),
                                int(variant)),
          "forces_raw")
    return F


def potentials_raw(R, L: float, lDeb: float, nseg: int = 0, device: int = -1, variant: int = 1):
    """U[i] = sum_{j != i} exp(-r/lDeb)/r inside L/2 (kernel 1 potential mode, stateless)."""
    R = np.ascontiguousarray(R, dtype=np.float64)
    N = R.shape[1]
    U = np.zeros(N)
    check(lib().mdqt_potentials_raw(N, float(L), float(lDeb), dptr(R), N, dptr(U), int(nseg), int(device),
                                    int(variant)),
          "potentials_raw")
    return U


def comm_unique_id() -> bytes:
    """a fresh RCCL unique id (rank 0 makes it; the launcher broadcasts it)"""
    buf = C.create_string_buffer(128)
    check(lib().mdqt_comm_unique_id(buf, 128), "comm_unique_id")
    return buf.raw


def comm_init_local(sims) -> None:
    """join the contexts of one process into an in-process group (tests on one GPU)"""
    arr = (C.c_void_p * len(sims))(*[s.h.value for s in sims])
    check(lib().mdqt_comm_init_local(arr, len(sims)), "comm_init_local")


class Simulation:
    """One MDQT system (or one rank's slab of it) resident on one MI355X."""

    def __init__(self, pump_program: int = 0, **params):
        """pump_program 1 / 2 / 3: start from that optical-pumping program's defaults
        (mdqt_default_params_pump) instead of SpeedUp's"""
        self.params = default_params_pump(pump_program, **params) if pump_program else default_params(**params)
        h = C.c_void_p()
        check(lib().mdqt_create(C.byref(self.params), C.byref(h)), "mdqt_create")
        self.h = h

    # ---- lifecycle ----
    def close(self):
        if getattr(self, "h", None):
            lib().mdqt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- constants / counters ----
    def const(self, name: str) -> float:
        return lib().mdqt_get_const(self.h, name.encode())

    @property
    def N(self) -> int:
        return lib().mdqt_get_N(self.h)

    @property
    def t(self) -> float:
        return lib().mdqt_get_time(self.h)

    @t.setter
    def t(self, v: float):
        check(lib().mdqt_set_time(self.h, float(v)))

    @property
    def qstep_index(self) -> int:
        return lib().mdqt_get_qstep_index(self.h)

    @qstep_index.setter
    def qstep_index(self, q: int):
        check(lib().mdqt_set_qstep_index(self.h, int(q)))

    @property
    def drand48_state(self) -> int:
        x = C.c_uint64()
        check(lib().mdqt_get_drand48_state(self.h, C.byref(x)))
        return x.value

    def counters(self):
        c0 = C.c_int(); cnt = C.c_uint(); e = C.c_double(); e0 = C.c_double()
        check(lib().mdqt_get_counters(self.h, C.byref(c0), C.byref(cnt), C.byref(e), C.byref(e0)))
        return dict(c0=c0.value, counter=cnt.value, Epot=e.value, Epot0=e0.value)

    # ---- state (host numpy <-> HBM) ----
    def init(self):
        check(lib().mdqt_init(self.h), "init")
        return self

    def set_state(self, R, V, psi, tPart, t):
        R = np.ascontiguousarray(R, dtype=np.float64)
        N = R.shape[1]
        V = np.ascontiguousarray(V, dtype=np.float64)
        psi = np.ascontiguousarray(psi, dtype=np.float64).reshape(N, NUM_STATES, 2)
        tPart = np.ascontiguousarray(tPart, dtype=np.float64)
        check(lib().mdqt_set_state(self.h, N, dptr(R), dptr(V), N, dptr(psi), dptr(tPart), float(t)),
              "set_state")

    def set_forces(self, F):
        F = np.ascontiguousarray(F, dtype=np.float64)
        check(lib().mdqt_set_forces(self.h, dptr(F), F.shape[1]), "set_forces")

    def get_state(self):
        N = self.N
        R = np.zeros((3, N)); V = np.zeros((3, N)); F = np.zeros((3, N))
        psi = np.zeros((N, NUM_STATES, 2)); tp = np.zeros(N); t = C.c_double()
        check(lib().mdqt_get_state(self.h, dptr(R), dptr(V), dptr(F), N, dptr(psi), dptr(tp),
                                   C.byref(t)), "get_state")
        return dict(R=R, V=V, F=F, psi=psi, tPart=tp, t=t.value)

    # ---- the reference's function seam ----
    def forces(self):
        check(lib().mdqt_forces(self.h), "forces")

    def step(self):
        check(lib().mdqt_step(self.h), "step")

    def qstep(self):
        check(lib().mdqt_qstep(self.h), "qstep")

    def substeps(self, n: int):
        check(lib().mdqt_substeps(self.h, int(n)), "substeps")

    def md_steps(self, n: int):
        check(lib().mdqt_md_steps(self.h, int(n)), "md_steps")

    def tag_spin_up(self):
        """measureSpinUps / tagParticles of the optical-pumping models: (tags[N], n_up)"""
        tags = np.zeros(self.N, dtype=np.int32)
        n = C.c_int()
        check(lib().mdqt_tag_spin_up(self.h, tags.ctypes.data_as(C.POINTER(C.c_int)), C.byref(n)),
              "tag_spin_up")
        return tags, n.value

    def Epotential(self) -> float:
        e = C.c_double()
        check(lib().mdqt_epotential(self.h, C.byref(e)), "Epotential")
        return e.value

    epotential = Epotential

    def potential_rows(self):
        """U_i, the per-ion pair-potential row sums Epotential() adds up (world 1; include/mdqt.h
        mdqt_potential_rows)"""
        import numpy as np
        U = np.zeros(self.N)
        check(lib().mdqt_potential_rows(self.h, U.ctypes.data_as(C.POINTER(C.c_double)), self.N), "potential_rows")
        return U

    def observables(self, kde: bool = True, pops: bool = True):
        o = np.zeros(7)
        P = np.zeros((3, NBINS)) if kde else None
        pp = np.zeros((self.N, 3)) if pops else None
        check(lib().mdqt_observables(self.h, dptr(o), dptr(P), dptr(pp)), "observables")
        return o, P, pp

    def partial_observables(self, vxAvg: float):
        o = np.zeros(5)
        P = np.zeros((3, NBINS))
        check(lib().mdqt_partial_observables(self.h, float(vxAvg), dptr(o), dptr(P)), "partial_observables")
        return o, P

    def setup_directories(self):
        check(lib().mdqt_setup_directories(self.h), "setup_directories")

    @property
    def save_directory(self) -> str:
        return lib().mdqt_save_directory(self.h).decode()

    def output(self):
        check(lib().mdqt_output(self.h), "output")

    def writeConditions(self, c0: int):
        check(lib().mdqt_write_conditions(self.h, int(c0)), "writeConditions")

    def readConditions(self, c0: int):
        check(lib().mdqt_read_conditions(self.h, int(c0)), "readConditions")

    write_conditions = writeConditions
    read_conditions = readConditions

    def run(self):
        check(lib().mdqt_run(self.h), "run")

    def run_pump(self):
        """the optical-pumping programs' main() (randomFrozenStartTag408Linear.cpp:981-1076;
        qt_model 1-3): mdqt_run_pump"""
        check(lib().mdqt_run_pump(self.h), "run_pump")

    def spin_up_list(self):
        """(tags[N], n_up) of the pumping run's measureSpinUps()"""
        tags = np.zeros(self.N, dtype=np.int32)
        n = C.c_int()
        check(lib().mdqt_get_spin_up_list(self.h, tags.ctypes.data_as(C.POINTER(C.c_int)), C.byref(n)),
              "spin_up_list")
        return tags, n.value

    def flush_files(self):
        """wait for the background file writers (mdqt_flush_files)"""
        check(lib().mdqt_flush_files(self.h), "flush_files")

    def set_option(self, name: str, value: int):
        check(lib().mdqt_set_option(self.h, name.encode(), int(value)), "set_option")

    # ---- streams / timing / sharding plumbing ----
    def set_stream(self, stream_handle: int | None):
        check(lib().mdqt_set_stream(self.h, C.c_void_p(stream_handle) if stream_handle else None))

    def synchronize(self):
        check(lib().mdqt_synchronize(self.h), "synchronize")

    def positions_device(self):
        p = C.c_void_p(); S = C.c_int()
        check(lib().mdqt_positions_device(self.h, C.byref(p), C.byref(S)))
        return p.value, S.value

    def slab_bounds(self):
        lo, hi = C.c_int(), C.c_int()
        check(lib().mdqt_slab_bounds(self.h, C.byref(lo), C.byref(hi)))
        return lo.value, hi.value

    def allgather_positions(self):
        check(lib().mdqt_allgather_positions(self.h), "allgather_positions")

    def allreduce_sum(self, buf):
        buf = np.ascontiguousarray(buf, dtype=np.float64)
        check(lib().mdqt_allreduce_sum(self.h, dptr(buf), buf.size), "allreduce_sum")
        return buf

    def comm_init(self, uid: bytes):
        check(lib().mdqt_comm_init(self.h, uid, len(uid)), "comm_init")

    def comm_size(self) -> int:
        """ranks of this context's communicator (ncclCommCount; 1 without one)"""
        n = C.c_int(0)
        check(lib().mdqt_comm_size(self.h, C.byref(n)), "comm_size")
        return n.value

    def enable_timing(self, period: int = 1, kinds: int = 3, offset: int | None = None):
        """bracket every `period`-th hot-kernel launch with HIP events (0/False: off); kinds:
        bit 0 force launches, bit 1 fused-substep launches, bit 2 the potential calls' block kernel, bit 3
        the force-call breakdown (force_breakdown); offset: which launch of each period (default
        period // 2)"""
        if offset is None:
            check(lib().mdqt_enable_timing_kinds(self.h, int(period), int(kinds)))
        else:
            check(lib().mdqt_enable_timing_at(self.h, int(period), int(kinds), int(offset)))

    CENSUS_CLASSES = ("skip_cut", "skip_tail", "ragged", "exact_image", "exact_uniform", "far_image",
                      "far_uniform", "vfar_image", "vfar_uniform", "ufar_uniform", "ufar32_uniform", "skip_sub",
                      "mid_image", "mid_uniform", "ufar_image")

    def force_census(self):
        """the Newton-3 block kernel's work by tile-pair class for the current positions (this rank's
        block pairs): {class: (lane_steps, ion_pairs)} (include/mdqt.h mdqt_force_census)"""
        n = len(self.CENSUS_CLASSES)
        out = (C.c_double * (2 * n))()
        check(lib().mdqt_force_census(self.h, out, 2 * n), "force_census")
        return {k: (out[i], out[n + i]) for i, k in enumerate(self.CENSUS_CLASSES)}

    def force_block_work(self):
        """the block kernel's evaluated lane-steps per block of this rank (numpy array; include/mdqt.h
        mdqt_force_block_work)"""
        import numpy as np
        nb = C.c_int()
        n = max(1, int(self.const("n3b_blocks")))
        out = np.zeros(n)
        check(lib().mdqt_force_block_work(self.h, out.ctypes.data_as(C.POINTER(C.c_double)), n, C.byref(nb)),
              "force_block_work")
        return out[:nb.value].copy()

    def force_jstep_balance(self):
        """the block kernel's J-step balance over a workgroup's 8 waves (diagnostic; include/mdqt.h
        mdqt_force_jstep_balance): {valu, valu_lockstep, jsteps, excess}"""
        out = (C.c_double * 11)()
        check(lib().mdqt_force_jstep_balance(self.h, out, 11), "force_jstep_balance")
        return {"valu": out[0], "valu_lockstep": out[1], "jsteps": int(out[2]),
                "excess": out[1] / out[0] if out[0] else None,
                "pairs_lockstep": out[4], "pairs_best_two_substeps": out[3], "row_floor": out[5],
                "excess_two_substeps": out[1] / out[0] * out[3] / out[4] if out[0] and out[4] else None,
                "excess_row_floor": out[5] / out[0] if out[0] else None,
                "excess_pairs_heavy_light": out[6] / out[0] if out[0] else None,
                "excess_pairs_q_7mq": out[7] / out[0] if out[0] else None,
                "excess_pairs_q_qp4": out[8] / out[0] if out[0] else None,
                "excess_pairs_per_jstep": out[9] / out[0] if out[0] else None,
                "excess_pairs_best_of_105": out[10] / out[0] if out[0] else None}

    def kernel_time_totals(self):
        """(force_ms, n_force_launches, substep_ms, n_substep_launches) since the last call"""
        a = C.c_double(); b = C.c_double(); na = C.c_int(); nb = C.c_int()
        check(lib().mdqt_kernel_time_totals(self.h, C.byref(a), C.byref(na), C.byref(b), C.byref(nb)))
        return a.value, na.value, b.value, nb.value

    def kernel_times(self):
        """{force_ms, n_force, substep_ms, n_substep, block_ms, n_block, pot_block_ms, n_pot_block} since
        the last call (block: the Newton-3 block kernel alone inside the timed force calls; pot_block: the
        same kernel in the timed potential calls, timing kinds bit 2; include/mdqt.h mdqt_kernel_times)"""
        out = (C.c_double * 8)()
        check(lib().mdqt_kernel_times(self.h, out, 8), "kernel_times")
        keys = ("force_ms", "n_force", "substep_ms", "n_substep", "block_ms", "n_block", "pot_block_ms", "n_pot_block")
        return {k: (int(out[i]) if k.startswith("n_") else out[i]) for i, k in enumerate(keys)}

    BREAKDOWN_KEYS = ("allgather", "sort_boxes", "plan", "block_kernel", "slot_reduce", "tail_pass",
                      "reduce_scatter", "forces_total")

    def force_breakdown(self):
        """the force-call breakdown (timing kinds bit 3, with bit 0): average ms per timed block-scheme
        force call of each stage, and the number of calls (include/mdqt.h mdqt_force_breakdown)"""
        out = (C.c_double * 9)()
        check(lib().mdqt_force_breakdown(self.h, out, 9), "force_breakdown")
        d = {k: out[i] for i, k in enumerate(self.BREAKDOWN_KEYS)}
        d["calls"] = int(out[8])
        return d


def tier_radius_model(N: int, L: float, lDeb: float, k: int, level: int, hi: float | None = None,
                      scale: float = 1.0, apriori: int = 0):
    """force_form_mode 1's radius of a pair-form tier and its bound, for given parameters, without a
    context or device (include/mdqt.h mdqt_tier_radius_model): level 1 far, 2 very far, 3 ultra far, 4
    ultra far in f32, 5 mid; hi the skip radius the model integrates to (default L/2); apriori 1: force_form_mode
    0's radius, 2: the a-priori cap the model takes"""
    r, b = C.c_double(), C.c_double()
    check(lib().mdqt_tier_radius_model(int(N), float(L), float(lDeb), int(k), int(level),
                                       float(L / 2 if hi is None else hi), float(scale), int(apriori),
                                       C.byref(r), C.byref(b)), "tier_radius_model")
    return r.value, b.value


__all__ = ["forces_raw", "potentials_raw", "tier_radius_model", "Simulation", "MdqtError", "default_params", "device_count", "slab", "NBINS", "NUM_STATES"]
