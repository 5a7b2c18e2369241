"""ctypes binding of libmdqt.so (the C ABIs declared in include/mdqt.h and include/mdmc.h).

The library is built in-tree (``python -m mdqtplasmasims_amd.build`` or ``__graft_entry__.build()``)
into ``mdqtplasmasims_amd/lib/libmdqt.so``.  There is no fallback: if the library is missing or
cannot be loaded, :func:`lib` raises, and every simulation call fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MDQT_LIB: an alternative build of the same library (kernel A/B experiments, tools/expt.sh)
LIB_PATH = os.environ.get("MDQT_LIB") or os.path.join(HERE, "lib", "libmdqt.so")
CLI_PATH = os.path.join(HERE, "bin", "mdqt")
MDMC_CLI_PATH = os.path.join(HERE, "bin", "mdmc")

_dp = C.POINTER(C.c_double)


class MdqtParams(C.Structure):
    """mirror of ``struct mdqt_params`` (include/mdqt.h)."""
    _fields_ = [
        ("Ge", C.c_double), ("tmax", C.c_double), ("density", C.c_double), ("sig0", C.c_double),
        ("Te", C.c_double), ("fracOfSig", C.c_double), ("detuning", C.c_double),
        ("detuningDP", C.c_double), ("Om", C.c_double), ("OmDP", C.c_double),
        ("N0", C.c_int), ("newRun", C.c_int), ("c0", C.c_int), ("sampleFreq", C.c_int),
        ("reNormalizewvFns", C.c_int), ("qt_enabled", C.c_int), ("rng_mode", C.c_int),
        ("seed", C.c_uint32), ("job", C.c_uint32), ("device", C.c_int), ("world_size", C.c_int),
        ("rank", C.c_int), ("force_segments", C.c_int), ("qt_model", C.c_int),
        ("saveDirectory", C.c_char * 256),
        ("tpumpreal", C.c_double), ("tstartV0", C.c_double),
    ]


class MdmcParams(C.Structure):
    """mirror of ``struct mdmc_params`` (include/mdmc.h)."""
    _fields_ = [
        ("N", C.c_int), ("kappa", C.c_double), ("Gamma", C.c_double), ("n", C.c_double),
        ("collisionFreq", C.c_double), ("monteCarloSteps", C.c_int), ("maxRStep", C.c_double),
        ("pairPairStep", C.c_double), ("timeStep", C.c_double), ("numPreRecordMDSteps", C.c_int),
        ("numVelAutoCorrsSteps", C.c_int), ("numInstantaneousAnisotropySteps", C.c_int),
        ("numReestablishEquilSteps", C.c_int), ("tempPercentDiff", C.c_double),
        ("applyForceAlongOneAxisOnly", C.c_int), ("beta", C.c_double),
        ("anisotropyEstablishmentTime", C.c_int), ("anisotropyFromForcesRelaxSteps", C.c_int),
        ("seed", C.c_uint32), ("job", C.c_uint32), ("device", C.c_int), ("force_kernel", C.c_int),
        ("qt_model", C.c_int), ("tpumpreal", C.c_double), ("detuning", C.c_double), ("Om", C.c_double),
        ("saveDirectory", C.c_char * 256),
    ]


_ip = C.POINTER(C.c_int)

# include/mdmc.h
MDMC_SIGNATURES = [
    ("mdmc_default_params", None, [C.POINTER(MdmcParams)]),
    ("mdmc_create", C.c_int, [C.POINTER(MdmcParams), C.POINTER(C.c_void_p)]),
    ("mdmc_destroy", None, [C.c_void_p]),
    ("mdmc_get_const", C.c_double, [C.c_void_p, C.c_char_p]),
    ("mdmc_init", C.c_int, [C.c_void_p]),
    ("mdmc_monte_carlo", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_longlong)]),
    ("mdmc_md_steps", C.c_int, [C.c_void_p, C.c_int]),
    ("mdmc_set_collision_freq", C.c_int, [C.c_void_p, C.c_double]),
    ("mdmc_set_laser_force", C.c_int, [C.c_void_p, C.c_int]),
    ("mdmc_pair_corr", C.c_int, [C.c_void_p, _dp, C.c_int, _ip]),
    ("mdmc_record_velocities", C.c_int, [C.c_void_p, C.c_int]),
    ("mdmc_autocorrelations", C.c_int, [C.c_void_p, _dp]),
    ("mdmc_set_velocity_store", C.c_int, [C.c_void_p, _dp]),
    ("mdmc_temperatures", C.c_int, [C.c_void_p, _dp]),
    ("mdmc_anisotropize", C.c_int, [C.c_void_p]),
    ("mdmc_tag_particles", C.c_int, [C.c_void_p, _ip]),
    ("mdmc_tagged_moments", C.c_int, [C.c_void_p, _dp]),
    ("mdmc_get_state", C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp]),
    ("mdmc_set_state", C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp]),
    ("mdmc_setup_directories", C.c_int, [C.c_void_p]),
    ("mdmc_save_directory", C.c_char_p, [C.c_void_p]),
    ("mdmc_run", C.c_int, [C.c_void_p, C.c_int]),
    ("mdmc_default_params_qt", C.c_int, [C.POINTER(MdmcParams), C.c_int]),
    ("mdmc_qsteps", C.c_int, [C.c_void_p, C.c_int]),
    ("mdmc_tag_qt", C.c_int, [C.c_void_p, _ip, _ip]),
    ("mdmc_tagged_moments_qt", C.c_int, [C.c_void_p, _dp, _dp]),
    ("mdmc_get_psi", C.c_int, [C.c_void_p, _dp]),
    ("mdmc_set_psi", C.c_int, [C.c_void_p, _dp]),
]

# (name, restype, argtypes) of every symbol include/mdqt.h declares
SIGNATURES = [
    ("mdqt_default_params", None, [C.POINTER(MdqtParams)]),
    ("mdqt_create", C.c_int, [C.POINTER(MdqtParams), C.POINTER(C.c_void_p)]),
    ("mdqt_destroy", None, [C.c_void_p]),
    ("mdqt_last_error", C.c_char_p, []),
    ("mdqt_device_count", C.c_int, []),
    ("mdqt_version", C.c_char_p, []),
    ("mdqt_get_const", C.c_double, [C.c_void_p, C.c_char_p]),
    ("mdqt_init", C.c_int, [C.c_void_p]),
    ("mdqt_get_N", C.c_int, [C.c_void_p]),
    ("mdqt_get_time", C.c_double, [C.c_void_p]),
    ("mdqt_set_time", C.c_int, [C.c_void_p, C.c_double]),
    ("mdqt_get_qstep_index", C.c_uint64, [C.c_void_p]),
    ("mdqt_set_qstep_index", C.c_int, [C.c_void_p, C.c_uint64]),
    ("mdqt_get_drand48_state", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    ("mdqt_get_counters", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint), _dp, _dp]),
    ("mdqt_set_state", C.c_int, [C.c_void_p, C.c_int, _dp, _dp, C.c_size_t, _dp, _dp, C.c_double]),
    ("mdqt_get_state", C.c_int, [C.c_void_p, _dp, _dp, _dp, C.c_size_t, _dp, _dp, _dp]),
    ("mdqt_set_forces", C.c_int, [C.c_void_p, _dp, C.c_size_t]),
    ("mdqt_forces", C.c_int, [C.c_void_p]),
    ("mdqt_step", C.c_int, [C.c_void_p]),
    ("mdqt_qstep", C.c_int, [C.c_void_p]),
    ("mdqt_substeps", C.c_int, [C.c_void_p, C.c_int]),
    ("mdqt_md_steps", C.c_int, [C.c_void_p, C.c_int]),
    ("mdqt_forces_raw", C.c_int, [C.c_int, C.c_double, C.c_double, _dp, C.c_size_t, _dp, C.c_int, C.c_int,
                                  C.c_int]),
    ("mdqt_potentials_raw", C.c_int, [C.c_int, C.c_double, C.c_double, _dp, C.c_size_t, _dp, C.c_int,
                                      C.c_int, C.c_int]),
    ("mdqt_epotential", C.c_int, [C.c_void_p, _dp]),
    ("mdqt_observables", C.c_int, [C.c_void_p, _dp, _dp, _dp]),
    ("mdqt_setup_directories", C.c_int, [C.c_void_p]),
    ("mdqt_save_directory", C.c_char_p, [C.c_void_p]),
    ("mdqt_output", C.c_int, [C.c_void_p]),
    ("mdqt_write_conditions", C.c_int, [C.c_void_p, C.c_int]),
    ("mdqt_read_conditions", C.c_int, [C.c_void_p, C.c_int]),
    ("mdqt_run", C.c_int, [C.c_void_p]),
    ("mdqt_run_pump", C.c_int, [C.c_void_p]),
    ("mdqt_get_spin_up_list", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("mdqt_default_params_pump", None, [C.POINTER(MdqtParams), C.c_int]),
    ("mdqt_flush_files", C.c_int, [C.c_void_p]),
    ("mdqt_tag_spin_up", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("mdqt_set_option", C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    ("mdqt_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("mdqt_get_stream", C.c_void_p, [C.c_void_p]),
    ("mdqt_synchronize", C.c_int, [C.c_void_p]),
    ("mdqt_slab", C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                            C.POINTER(C.c_int)]),
    ("mdqt_positions_device", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int)]),
    ("mdqt_partial_observables", C.c_int, [C.c_void_p, C.c_double, _dp, _dp]),
    ("mdqt_slab_bounds", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("mdqt_set_counters", C.c_int, [C.c_void_p, C.c_int, C.c_uint, C.c_double, C.c_double]),
    ("mdqt_comm_unique_id", C.c_int, [C.c_char_p, C.c_size_t]),
    ("mdqt_comm_init", C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    ("mdqt_comm_init_local", C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    ("mdqt_comm_size", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("mdqt_allgather_positions", C.c_int, [C.c_void_p]),
    ("mdqt_allreduce_sum", C.c_int, [C.c_void_p, _dp, C.c_size_t]),
    ("mdqt_force_census", C.c_int, [C.c_void_p, _dp, C.c_int]),
    ("mdqt_kernel_time_totals", C.c_int, [C.c_void_p, _dp, C.POINTER(C.c_int), _dp, C.POINTER(C.c_int)]),
    ("mdqt_kernel_times", C.c_int, [C.c_void_p, _dp, C.c_int]),
    ("mdqt_force_breakdown", C.c_int, [C.c_void_p, _dp, C.c_int]),
    ("mdqt_potential_rows", C.c_int, [C.c_void_p, _dp, C.c_int]),
    ("mdqt_force_jstep_balance", C.c_int, [C.c_void_p, _dp, C.c_int]),
    ("mdqt_tier_radius_model", C.c_int, [C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_double, C.c_double,
                                         C.c_int, _dp, _dp]),
    ("mdqt_force_block_work", C.c_int, [C.c_void_p, _dp, C.c_int, C.POINTER(C.c_int)]),
    ("mdqt_enable_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("mdqt_enable_timing_kinds", C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    ("mdqt_enable_timing_at", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
]

_lib = None


class MdqtError(RuntimeError):
    pass


def lib():
    """Load libmdqt.so (raises if it has not been built: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MdqtError(f"{LIB_PATH} not built: run `python -m mdqtplasmasims_amd.build` "
                            "(the MDQT engine has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES + MDMC_SIGNATURES:
            try:
                f = getattr(L, name)
            except AttributeError:
                # an older experiment build (MDQT_LIB, kernel A/B) may predate an entry point; the
                # product library must export every one (tests/test_capi.py)
                if "MDQT_LIB" not in os.environ:
                    raise
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().mdqt_last_error().decode(errors="replace")
        raise MdqtError(f"{what}: {msg}" if what else msg)


def dptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None
