#!/usr/bin/env python3
"""Benchmark of the MDQT hot path on MI355X (one JSON line on rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c5] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A "step" is one MD step of the reference time loop (SpeedUp:1369-1377): forces() once, then
plasmaToQuantumTimestepRatio (= 25 at density 2) x (step(); qstep()), all on the GPU, state
resident in HBM.  The metric is BASELINE.json's: particle-steps/s with QT on, reported in
particle-qsteps/s (N x quantum substeps / wall time).

Workload at N=1 is BASELINE.json configs[1] (C2): N0=3500 full MDQT, detuning=-1, Om=1,
density 2 (realised N=3573 for seed 12346).  Synthetic inputs exactly as the reference's init()
(drand48 seeded 12345+job).  With N>1 GPUs C2 does not shard (~10 µs
of force per MD step), so each rank runs an independent replica (job = rank+1), like the
reference's SLURM array (exampleSlurmFile.slurm:3): "replicas only", weak scaling.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFS = 78.6       # MI355X fp64 vector (spec), SURVEY §8d
B_Q_PER_ION = 520.0        # algorithmic bytes per ion per fused-substep launch
F_Q_PER_QSTEP = 1750.0     # fp64 flop per particle-qstep
W_F_PER_PAIR = 30.0        # fp64 flop per distinct pair
FP32_PEAK_TFS = 157.3      # MI355X fp32 vector (spec): the roof of the block kernel's f32 ultra-far form
F32_TIERS = ("ufar32_uniform",)   # census classes whose pair terms run in f32 (mdqt_forces.hip n3b_group_uf32)

METRIC = "particle-steps/sec (MD+QT) at N=3.5k and N=1M; 1/2/4/8-GPU scaling"
LINE_MAX_BYTES = 8192      # the driver parses the last stdout line; VERDICT r04 item 1

CONFIGS = {
    # name: (params, qt, description)
    "c2": (dict(N0=3500), 1, "C2: N0=3500 full MDQT, detuning=-1, Om=1, density=2, fp64"),
    "c1": (dict(N0=500, Ge=0.1), 0, "C1: N0=500 Yukawa OCP MD-only, Ge=0.1"),
    "c3": (dict(N0=100000, Ge=1.0 / 12), 0, "C3: N0=100000 MD-only, kappa=0.5"),
    "c4": (dict(N0=1000000, Ge=1.0 / 12), 0, "C4: N0=1000000 MD-only, kappa=0.5"),
    "c5": (dict(N0=250000, detuningDP=1.0), 1, "C5: N0=250000 full MDQT, detuningDP=+1"),
    # BASELINE.json north_star: "particle-steps/sec at N=3 500 and N=1 000 000 with QT on"
    "c1m": (dict(N0=1000000), 1, "N0=1000000 full MDQT (C2's laser parameters, density 2)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--sharded-config", default="c5", choices=["none", "c3", "c5", "c4", "c1m"])
    ap.add_argument("--million-config", default="c1m", choices=["none", "c1m", "c4"],
                    help="the N=1M line of the metric (QT on), one system sharded over all ranks")
    ap.add_argument("--million-steps", type=int, default=2)
    ap.add_argument("--md-only-config", default="c3,c4",
                    help="comma-separated MD-only lines (force-kernel FP64 roofline runs; BASELINE configs[2] = "
                         "C3, configs[3] = C4), or none")
    ap.add_argument("--no-e2e-line", action="store_true",
                    help="skip the end-to-end line (reference cadence: output() every sampleFreq MD steps)")
    ap.add_argument("--e2e-md-steps", type=int, default=400)
    ap.add_argument("--e2e-large", default="c5,c1m",
                    help="comma-separated large configs with an end-to-end line (mdqt_run, output every 40 MD "
                         "steps: 40 more MD steps and one output), or none")
    ap.add_argument("--no-replicas-line", action="store_true",
                    help="skip the jobs-per-GPU line (k independent C2 jobs sharing one GPU)")
    ap.add_argument("--secondary-deadline", type=float, default=420.0,
                    help="seconds allowed for all secondary line items together")
    ap.add_argument("--sharded-in-child", type=int, default=-1,
                    help="run the sharded lines in child processes (own RCCL group) so that a fault "
                         "there cannot take the headline line with it: 1 yes, 0 no, -1 auto (world > 1)")
    ap.add_argument("--child-sharded", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-steps", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--sharded-steps", type=int, default=3)
    ap.add_argument("--qt-math", type=int, default=2, choices=[0, 1, 2],
                    help="0: the reference's exact QT operations, 1: FMA-contracted, 2: reassociated "
                         "(option qt_math, the library default)")
    ap.add_argument("--timed-launch", default="mid", choices=["mid", "first", "last"],
                    help="which MD step of the timed window carries the one event-timed launch")
    ap.add_argument("--overlap", type=int, default=0, choices=[0, 1],
                    help="1: each MD step's QT launch overlaps its force launch (option overlap; "
                         "measured slower, DESIGN.md §8); 0: the sequential order (library default)")
    ap.add_argument("--no-pump-lines", action="store_true",
                    help="skip the optical-pumping model lines (SURVEY §8(f)3)")
    ap.add_argument("--no-mcmd-lines", action="store_true",
                    help="skip the Monte-Carlo + MD analytics program line (SURVEY §8(f)4)")
    ap.add_argument("--timing-period", type=int, default=0,
                    help="bracket every k-th kernel launch of the timed region with HIP events "
                         "(0: the steps, i.e. one sampled launch of each kernel, mid-window)")
    return ap.parse_args()


def md_only_configs(spec):
    """--md-only-config: 'none' or a comma-separated list of MD-only configs (c1, c3, c4)"""
    if spec in ("", "none"):
        return []
    cfgs = [c.strip() for c in spec.split(",") if c.strip()]
    for c in cfgs:
        if c not in CONFIGS or CONFIGS[c][1]:
            raise SystemExit(f"bench.py: --md-only-config: {c} is not an MD-only config (c1, c3, c4)")
    return cfgs


def kernel_source_hash():
    """sha256 (16 hex) of the kernel sources (mdqtplasmasims_amd/csrc: .hip .hpp .cpp Makefile): a PMC
    summary records the hash of the tree it was measured on, and the bench uses its counters only when
    the hash matches its own tree — a kernel change makes the committed traffic figure stale, and the
    line then says so instead of quoting it"""
    import hashlib
    d = os.path.join(ROOT, "mdqtplasmasims_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".hpp", ".cpp")) or f == "Makefile":
            h.update(f.encode())
            with open(os.path.join(d, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def latest_pmc_file():
    """the newest committed C2 PMC summary (profiles/r<round><letter>_c2_pmc.json)"""
    d = os.path.join(ROOT, "profiles")
    fs = sorted(f for f in os.listdir(d) if f.endswith("_c2_pmc.json") and f.startswith("r"))
    return os.path.join(d, fs[-1]) if fs else None


def pmc_traffic(kernel_prefix, path=None):
    """HBM-side bytes per launch of the kernel (FETCH_SIZE + WRITE_SIZE, separate rocprofv3 --pmc
    passes of the same C2 workload, kB -> B) from the newest committed PMC summary, corrected by the
    calibration factors that summary carries (tools/fetch_calib.hip: FETCH_SIZE / known bytes of the
    kernel's own access pattern).  The production instance (the most dispatched one of the kernel
    family) is taken.  Returns (bytes or None, source dict): None when the summary was measured on
    other kernel sources than this tree's (its src_hash), or has no such kernel."""
    path = path or latest_pmc_file()
    src = {"file": os.path.relpath(path, ROOT) if path else None, "src_hash": kernel_source_hash()}
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, TypeError):
        return None, dict(src, status="no PMC summary")
    meta = d.get("_meta", {})
    src["measured_src_hash"] = meta.get("src_hash")
    if meta.get("src_hash") != src["src_hash"]:
        return None, dict(src, status="stale: measured on other kernel sources")
    best, name = None, None
    for k, v in d.items():
        if k == "_meta":
            continue
        short = k.split("(")[0].replace("void ", "").replace("mdqt::", "")
        if short.startswith(kernel_prefix) and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            if best is None or v.get("dispatches", 0) > best.get("dispatches", 0):
                best, name = v, short
    if best is None:
        return None, dict(src, status="kernel not in the summary")
    cf = meta.get("fetch_factor", 1.0)            # FETCH_SIZE / true bytes for this access pattern
    cw = meta.get("write_factor", 1.0)
    src.update(status="ok", instance=name, fetch_kB=best["FETCH_SIZE"], write_kB=best["WRITE_SIZE"],
               fetch_factor=cf, write_factor=cw)
    if all(k in best for k in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES")) and best["SQ_WAVES"]:
        # the launch's issue picture from the same PMC summary: per wave, VALU and SALU instructions and
        # its lifetime (SQ_WAVE_CYCLES counts quad-cycles); one instruction per wave issues every 4
        # cycles at most, so (VALU + SALU) x 4 / lifetime is the wave's issue-slot occupancy
        w = best["SQ_WAVES"]
        life = best["SQ_WAVE_CYCLES"] * 4.0 / w
        src["issue"] = {"valu_per_wave": best["SQ_INSTS_VALU"] / w, "salu_per_wave": best["SQ_INSTS_SALU"] / w,
                        "wave_cycles": life,
                        "issue_slot_frac": (best["SQ_INSTS_VALU"] + best["SQ_INSTS_SALU"]) / w * 4.0 / life}
    return (best["FETCH_SIZE"] / cf + best["WRITE_SIZE"] / cw) * 1024.0, src


def cpu_threads():
    """the GPU box's CPU share (16 per GPU; os.cpu_count() reports the whole machine there)"""
    return max(1, min(16, os.cpu_count() or 1))


def cpu_baseline(params, qt, seconds, seed, job):
    """The oracle (CPU restatement, race-free OpenMP) on a bounded sample of the same workload, at
    the box's CPU share (16 threads) and on one thread (BASELINE.md §3 asks for both)."""
    from oracle import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()

    def timed(threads, budget, cap):
        o = O.OracleSim(rng_mode=1, nthreads=threads, qt_enabled=qt, seed=seed, job=job, **params).init()
        ratio = int(o.const("plasmaToQuantumTimestepRatio"))
        o.md_steps(1)                              # warm
        n, t0 = 0, time.perf_counter()
        while True:
            o.md_steps(1)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= cap:
                break
        N = o.N
        o.close()
        return N * ratio * n / el, n, ratio, N, el

    threads = cpu_threads()
    rate, n, ratio, N, el = timed(threads, seconds, 400)
    r1, n1, _, _, el1 = timed(1, max(2.0, seconds / 3), 100)
    out = {"value": rate, "unit": "particle-qsteps/s", "cores": threads, "kind": "port",
           "sample": f"{n} MD steps x {ratio} qsteps of the same workload (N={N}), oracle C "
                     f"restatement, OpenMP {threads} threads, {el:.1f} s",
           "single_thread": {"value": r1, "unit": "particle-qsteps/s", "cores": 1,
                             "sample": f"{n1} MD steps x {ratio} qsteps, 1 thread, {el1:.1f} s"},
           "calibration": None}
    cal = calibration_file()
    if cal:                                        # the port against the reference itself
        with open(cal) as f:
            c = json.load(f)
        k = c["threads"]["1"]["oracle_over_reference"]
        out["calibration"] = {
            "file": os.path.relpath(cal, ROOT), "oracle_over_reference_1_thread": k,
            "reference_1_thread": c["threads"]["1"]["reference_particle_qsteps_per_s"],
            "oracle_1_thread_same_container": c["threads"]["1"]["oracle_particle_qsteps_per_s"],
            "reference_equivalent_on_this_host_1_thread": r1 / k,
            "note": "the reference SpeedUp's own 1-thread rate (BASELINE.md 2, SURVEY App. B-3) and the oracle's on "
                    "the same container and workload: the oracle is k x faster, so the reference would run about "
                    "single_thread / k here"}
    return out


def calibration_file():
    """the newest committed CPU calibration (profiles/r<round>_cpu_calibration.json, tools/cpu_calibration.py)"""
    d = os.path.join(ROOT, "profiles")
    fs = sorted(f for f in os.listdir(d) if f.endswith("_cpu_calibration.json") and f.startswith("r"))
    return os.path.join(d, fs[-1]) if fs else None


def cpu_baseline_large(cfg, seconds=6.0):
    """CPU baseline of a large line (C3 / C5 / N = 1M; BASELINE.md §3: time a part of one MD interval
    and extrapolate).  The race-free CPU restatement computes owner rows (each pair from both
    sides: N(N-1) pair terms per forces()): forces_rows over a block of rows, timed, scaled to all N
    rows; with QT on, plus one MD interval of qsteps on a sample of ions (ions are independent
    between force calls), scaled to N.  Inputs: the reference's init() positions are replaced by
    uniform positions of the same N and box (the cost does not depend on them)."""
    import numpy as np
    from oracle import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    params, qt, desc = CONFIGS[cfg]
    threads = cpu_threads()
    o = O.OracleSim(rng_mode=1, nthreads=threads, qt_enabled=qt, seed=12346, job=1, **params)
    L, lDeb, ratio = o.const("L"), o.const("lDeb"), int(o.const("plasmaToQuantumTimestepRatio"))
    N = int(params["N0"])
    R = np.random.default_rng(5).uniform(0, L, (3, N))
    rows = max(threads * 4, int(threads * 3.7e7 * seconds / 2 / N))   # ~half the budget
    rows = min(rows, N)
    t0 = time.perf_counter()
    O.forces_rows(R, 0, rows, L, lDeb, nthreads=threads)
    t_rows = time.perf_counter() - t0
    t_force = t_rows * N / rows
    t_qt, nq = 0.0, 0
    if qt:
        nq = min(N, 20000)
        V = np.zeros((3, nq))
        psi = np.zeros((nq, 12, 2)); psi[:, 0, 0] = 1.0
        o.set_state(R[:, :nq], V, psi, np.zeros(nq), 0.0)
        o.set_forces(np.zeros((3, nq)))
        t0 = time.perf_counter()
        o.substeps(ratio)
        t_qt = (time.perf_counter() - t0) * N / nq
    o.close()
    per_md_step = t_force + t_qt
    units = ratio if qt else 1
    return {"value": N * units / per_md_step, "unit": "particle-qsteps/s" if qt else "particle-MD-steps/s",
            "cores": threads, "kind": "port", "s_per_md_step": per_md_step,
            "sample": f"forces_rows over {rows} of {N} rows ({rows * (N - 1):.3g} pair terms, {t_rows:.1f} s)"
                      + (f" + {ratio} qsteps on {nq} ions" if qt else "")
                      + f", extrapolated to one MD step of N={N}; oracle C restatement, OpenMP {threads} threads"}


def child_main(args):
    """one rank of a sharded line in its own process and RCCL group (see sharded_in_children)"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    res = sharded_run(args.child_sharded, args.child_steps, rank, world, local, dist, barrier)
    if rank == 0:
        print("CHILD_JSON " + json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


_CHILD_PORT_OFFSET = [0]


def sharded_in_children(cfg, steps, rank, world, timeout):
    """Every rank starts one child process that runs the sharded line with the other ranks'
    children (a fresh RCCL group on another port); the parent only waits.  A child that faults
    or hangs costs this line only (reported in secondary_errors), never the headline."""
    import subprocess
    _CHILD_PORT_OFFSET[0] += 1
    env = dict(os.environ)
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)       # the child group runs its own store
    env["MASTER_ADDR"] = env.get("MASTER_ADDR", "127.0.0.1")
    env["MASTER_PORT"] = str(int(env.get("MASTER_PORT", "29500")) + 97 + _CHILD_PORT_OFFSET[0])
    env.setdefault("RANK", str(rank)); env.setdefault("WORLD_SIZE", str(world))
    env.setdefault("LOCAL_RANK", os.environ.get("LOCAL_RANK", "0"))
    cmd = [sys.executable, os.path.abspath(__file__), "--child-sharded", cfg, "--child-steps", str(steps)]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        raise RuntimeError(f"sharded child did not finish within {timeout:.0f} s")
    if r.returncode != 0:
        raise RuntimeError(f"sharded child exited {r.returncode}: {r.stderr.strip()[-400:]}")
    if rank != 0:
        return None
    for line in r.stdout.splitlines():
        if line.startswith("CHILD_JSON "):
            return json.loads(line[len("CHILD_JSON "):])
    raise RuntimeError("sharded child printed no result")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_launch_command(gpus, argv, env):
    """The command that starts the `gpus` rank processes of `bench.py --gpus N` when no launcher did
    (no WORLD_SIZE in the environment): torch.distributed.run, one process per GPU, on 127.0.0.1.
    None when this process already is a rank (or N = 1)."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env):
    """--gpus N must be the launcher's world size: a run that silently measures fewer GPUs than it
    was asked for is an error."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return world


def main():
    t_start = time.perf_counter()
    args = parse()
    if args.child_sharded:
        return child_main(args)
    # `python bench.py --gpus N` without a launcher: start the N ranks here, before this process
    # touches the GPU (no HIP call has been made yet), and exit with their status
    cmd = rank_launch_command(args.gpus, sys.argv[1:], os.environ)
    if cmd is not None:
        import subprocess
        print(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd[:6])} ...", file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd).returncode)
    world = check_world(args.gpus, os.environ)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    comm_size = 1
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        comm_size = dist.get_world_size()
        if comm_size != args.gpus:
            raise SystemExit(f"bench.py: the RCCL group has {comm_size} ranks, --gpus {args.gpus}")

    import mdqtplasmasims_amd as M
    params, qt, desc = CONFIGS[args.config]
    job = rank + 1
    sim = M.Simulation(device=local, seed=12345 + job, job=job, qt_enabled=qt, **params).init()
    sim.set_option("qt_math", args.qt_math)
    sim.set_option("overlap", args.overlap)
    N = sim.N
    ratio = int(sim.const("plasmaToQuantumTimestepRatio"))
    sim.md_steps(args.warmup)
    sim.synchronize()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    # sparse HIP-event sampling of the dominant kernel inside the timed region: one launch by
    # default, in the middle of the window (an event-timed launch costs its MD step a few us of
    # event handling — kernel trace: gaps of 4.4 / 7.8 / 4.4 us around a timed force + QT pair,
    # none elsewhere); the other kernel is timed in a short window after it
    dom = 2 if qt else 1                           # kinds bit: 1 force, 2 fused substeps
    if args.timing_period > 0 or args.timed_launch == "mid":
        sim.enable_timing(args.timing_period if args.timing_period > 0 else max(2, args.steps), dom)
    else:                                          # one launch: the window's first or last MD step
        sim.enable_timing(args.steps + 1, dom, 0 if args.timed_launch == "first" else args.steps - 1)
    t0 = time.perf_counter()
    sim.md_steps(args.steps)
    barrier()                                      # torch.cuda.synchronize: every stream of the device
    el = time.perf_counter() - t0
    f_ms, nf, s_ms, ns = sim.kernel_time_totals()
    sim.enable_timing(4, 3 - dom)                  # the other kernel, outside the timed region
    sim.md_steps(8)
    f2, nf2, s2, ns2 = sim.kernel_time_totals()
    sim.enable_timing(False)
    if dom == 2:
        f_ms, nf = f2, nf2
    else:
        s_ms, ns = s2, ns2

    tt = torch.tensor([el, float(N), f_ms, s_ms], dtype=torch.float64, device="cuda")
    if world > 1:
        mx = tt.clone(); dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone(); dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el_max, n_tot = float(mx[0]), float(sm[1])
    else:
        el_max, n_tot = el, float(N)

    if rank == 0:
        value = n_tot * ratio * args.steps / el_max
        # roofline of the dominant kernel (per-launch averages from the HIP events above)
        f_avg = f_ms / max(nf, 1) * 1e-3
        s_avg = s_ms / max(ns, 1) * 1e-3
        if qt:
            # substeps per fused launch: the MD interval split at MAXSUB = 32 (mdqt_internal.hpp)
            launches = -(-ratio // 32)
            nsub_per_launch = ratio / launches
            # B_q = 520 B per particle-QSTEP; one fused launch processes N x nsub
            # particle-qsteps, so its algorithmic bytes are 520 N nsub (the contract's "per-unit figure
            # x units per launch").  The launch keeps the state in registers across its substeps, so
            # the bytes it must move (compulsory) are 520 N once — the PMC traffic is measured against
            # those; and the roof that binds it is neither: FP64 VALU issue, the
            # line's roofline, with F_q = 1.75 kflop per particle-qstep.
            qsteps_launch = N * nsub_per_launch
            bytes_launch = B_Q_PER_ION * qsteps_launch
            ach = bytes_launch / s_avg / 1e9
            compulsory = B_Q_PER_ION * N
            flops = F_Q_PER_QSTEP * qsteps_launch
            kname = "k_substeps_lanes" if N < 98304 else "k_substeps_r"
            traffic, tsrc = pmc_traffic(kname)
            kinst = tsrc.get("instance")
            fp64 = flops / s_avg / 1e12
            # the roof that binds a register-fused launch is FP64 VALU issue (VERDICT r04
            # item 2): frac = 1,750 flop x particle-qsteps / launch time / 78.6 TF.  Beside it the HBM
            # figures: 8(d)'s 520 B per particle-qstep (a virtual rate for a fused launch), the PMC
            # traffic, and the compulsory 520 B per ion once.
            roof = {"bound": "fp64", "achieved": fp64, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": fp64 / FP64_PEAK_TFS, "traffic": traffic,
                    "kernel": f"{kinst or kname} (fused {nsub_per_launch:g} x step+qstep)",
                    "avg_launch_us": s_avg * 1e6, "flop_per_launch": flops,
                    "algorithmic_unit": f"{F_Q_PER_QSTEP:g} flop per particle-qstep x {qsteps_launch:.0f} "
                                        "particle-qsteps per launch (SURVEY 8d)",
                    "hbm_frac_8d": ach / HBM_PEAK_GBS,
                    "traffic_frac": traffic / s_avg / 1e9 / HBM_PEAK_GBS if traffic else None,
                    "compulsory_hbm_frac": compulsory / s_avg / 1e9 / HBM_PEAK_GBS,
                    "hbm_8d": {"achieved_GBs": ach, "bytes_per_launch": bytes_launch,
                               "unit": f"{B_Q_PER_ION:g} B per particle-qstep (SURVEY 8d)",
                               "compulsory_bytes_per_launch": compulsory},
                    "traffic_source": tsrc}
        else:
            pairs = N * (N - 1) / 2.0
            flops = W_F_PER_PAIR * pairs
            ach = flops / f_avg / 1e12
            roof = {"bound": "fp64", "achieved": ach, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": ach / FP64_PEAK_TFS, "traffic": None, "kernel": "forces() (Newton-3 tiles)",
                    "avg_launch_us": f_avg * 1e6,
                    "hbm_frac_8d": (24.0 * 2 * N) / f_avg / 1e9 / HBM_PEAK_GBS}
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "particle-qsteps/s",
            "n_gpus": world,
            "comm_size": comm_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference init(): drand48 positions + random S superposition, seed 12345+job)",
            "config": {"workload": desc, "N": N, "md_steps": args.steps, "qsteps_per_md_step": ratio,
                       "particle_md_steps_per_s": value / ratio,
                       "parallelism": ("replicas: one independent C2 system per GPU (job = rank + 1, like the "
                                       "reference's SLURM array); not one sharded system — that is the "
                                       "'sharded' / 'sharded_1m' lines") if world > 1 else "single",
                       "rng": "philox4x32-10", "kernel_ms": {"force_total": f_ms, "force_launches": nf,
                                                            "substeps_total": s_ms, "substep_launches": ns,
                                                            "timed_in_window": "substeps" if dom == 2 else "force",
                                                            "other_kernel": "8 MD steps after the window"}},
            "roofline": roof,
            "cpu_baseline": None,
            "timed_region_s": el_max,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(params, qt, args.cpu_seconds, 12345 + job, job)
        if world == 1 and not args.no_pump_lines:
            out["pump_models"] = pump_lines(local)
        if world == 1 and not args.no_mcmd_lines:
            out["mcmd"] = mcmd_line(local, cpu=not args.no_cpu_baseline)
    sim.close()
    # The secondary line items below run after the headline number is final.  A watchdog on every
    # rank bounds them: if one of them fails or does not finish in time, rank 0 prints the line
    # with what it has (and the reason) and every rank leaves, so the headline is never lost.
    out = out if rank == 0 else None
    dog = Watchdog(args.secondary_deadline, rank, out, t_start)
    if not args.no_replicas_line:
        dog.run("jobs_per_gpu", lambda: replicas_line(local, args.config))
    if world == 1 and not args.no_e2e_line:
        dog.run("end_to_end", lambda: end_to_end_line(local, args.config, args.e2e_md_steps))
    if world == 1 and not args.no_e2e_line and args.e2e_large != "none":
        for cfg in args.e2e_large.split(","):
            name = "end_to_end_" + ("1m" if cfg == "c1m" else cfg)
            dog.run(name, lambda cfg=cfg: end_to_end_line(local, cfg, 40, base=40, warm=False))
    # one large system sharded over all ranks (RCCL all-gather / reduce-scatter per MD step)
    in_child = args.sharded_in_child == 1 or (args.sharded_in_child == -1 and world > 1)

    def sharded(cfg, steps):
        if in_child:
            try:
                return sharded_in_children(cfg, steps, rank, world, timeout=150.0)
            finally:
                if world > 1:
                    dist.barrier()
        return sharded_run(cfg, steps, rank, world, local, dist, barrier)

    cpu_large = world == 1 and not args.no_cpu_baseline

    def with_cpu(cfg, res):
        if cpu_large and rank == 0 and res is not None:
            res["cpu_baseline"] = cpu_baseline_large(cfg)
        return res

    for cfg in md_only_configs(args.md_only_config):
        dog.run("md_only_" + cfg, lambda cfg=cfg: with_cpu(cfg, sharded(cfg, args.sharded_steps)))
    if args.sharded_config != "none":
        dog.run("sharded", lambda: with_cpu(args.sharded_config, sharded(args.sharded_config, args.sharded_steps)))
    if args.million_config != "none":
        dog.run("sharded_1m", lambda: with_cpu(args.million_config, sharded(args.million_config, args.million_steps)))
    dog.finish()
    if rank == 0:
        emit(out, t_start)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


PUMP_MODELS = [
    (1, dict(Om=0.7, detuning=-2.5), "408 nm linear pumping, 7 levels (randomFrozenStartTag408Linear.cpp)"),
    (2, dict(Om=2.0, detuning=0.0), "408 nm quad pumping, 7 levels (randomFrozenStartTag408Quad.cpp)"),
    (3, dict(Om=1.3, detuning=-1.0), "422 nm linear pumping, 5 levels (randomFrozenStartTag422Linear.cpp)"),
]


def pump_lines(local, steps=100):
    """the optical-pumping QT models on the C2 system: MD + pump qsteps"""
    import torch
    import mdqtplasmasims_amd as M
    res = []
    for model, kw, desc in PUMP_MODELS:
        sim = M.Simulation(device=local, N0=3500, seed=12346, job=1, qt_model=model, **kw).init()
        ratio = int(sim.const("plasmaToQuantumTimestepRatio"))
        sim.md_steps(10)
        sim.synchronize()
        t0 = time.perf_counter()
        sim.md_steps(steps)
        sim.synchronize()
        el = time.perf_counter() - t0
        res.append({"qt_model": model, "workload": desc + ", N0=3500, density 2", "N": sim.N,
                    "md_steps": steps, "ms_per_md_step": el / steps * 1e3,
                    "value": sim.N * ratio * steps / el, "unit": "particle-qsteps/s"})
        sim.close()
    torch.cuda.synchronize()
    return res


def mcmd_line(local, cpu=True, mc_steps=20000, md_steps=2000):
    """MonteCarloFollowedByMDAndTempAnisotropy.cpp at its own size, N = 4096:
    Metropolis steps/s, MD steps/s (collisionless and collisional), the analytics, and the whole
    main() estimated from the stage rates; beside it the reference build (oracle/_ref) on 1 core."""
    import tempfile
    import numpy as np
    from mdqtplasmasims_amd import mdmc
    tmp = tempfile.mkdtemp(prefix="mcmd_bench_")
    e = mdmc.MonteCarloMD(device=local, seed=3, saveDirectory=tmp + "/")
    p = e.p
    e.init()
    e.monte_carlo(1000)
    t0 = time.perf_counter(); acc = e.monte_carlo(mc_steps); mc_s = time.perf_counter() - t0
    e.md_steps(50)
    rates = {}
    for cf in (0.0, 0.25):
        e.set_collision_freq(cf)
        t0 = time.perf_counter(); e.md_steps(md_steps); rates[cf] = md_steps / (time.perf_counter() - t0)
    t0 = time.perf_counter(); e.pair_corr(); g_ms = (time.perf_counter() - t0) * 1e3
    vs = np.random.default_rng(1).normal(0, 0.5, (3, e.N, e.T))
    e.set_velocity_store(vs)
    e.autocorrelations()
    t0 = time.perf_counter(); e.autocorrelations(); ac_ms = (time.perf_counter() - t0) * 1e3
    e.close()
    mc_rate = mc_steps / mc_s
    nest = round(.8 * p.anisotropyEstablishmentTime * np.sqrt(p.n) / p.timeStep)
    n_free = p.numVelAutoCorrsSteps + p.numInstantaneousAnisotropySteps + nest + p.anisotropyFromForcesRelaxSteps
    n_coll = p.numPreRecordMDSteps + p.numReestablishEquilSteps
    est = p.monteCarloSteps / mc_rate + n_free / rates[0.0] + n_coll / rates[0.25] + ac_ms / 1e3 \
        + (p.monteCarloSteps // 10000 + p.numVelAutoCorrsSteps // 100) * g_ms / 1e3
    line = {"workload": "MonteCarloFollowedByMDAndTempAnisotropy.cpp main(): N=4096, kappa=0.5, Gamma=3 "
                        "(200000 MC steps, 8712 MD steps, g(r), 4 autocorrelations over 2500 steps)",
            "N": e.N, "mc_steps_per_s": mc_rate, "mc_acceptance": acc / mc_steps,
            "md_steps_per_s": rates[0.0], "md_collisional_steps_per_s": rates[0.25],
            "md_particle_steps_per_s": rates[0.0] * e.N,
            "pair_corr_ms": g_ms, "autocorrelations_ms": ac_ms, "main_estimate_s": est,
            "cpu_baseline": None}
    if cpu:
        from oracle import oracle as O
        if O.ref_available():
            r = O.RefMCMD(seed=3, save_directory=tmp + "/")
            r.init()
            t0 = time.perf_counter(); r.monte_carlo(2000); rmc = 2000 / (time.perf_counter() - t0)
            t0 = time.perf_counter(); r.md_steps(3); rmd = 3 / (time.perf_counter() - t0)
            rest = p.monteCarloSteps / rmc + (n_free + n_coll) / rmd
            line["cpu_baseline"] = {"kind": "reference", "cores": 1, "mc_steps_per_s": rmc, "md_steps_per_s": rmd,
                                    "main_estimate_s": rest,
                                    "sample": "the reference's MonteCarloStep x2000 and MDStep x3 "
                                              "(oracle/_ref/libmdref.so, 1 thread)"}
    line["qt_tagging"] = qtt_line(local)
    return line


def qtt_line(local, steps=10):
    """MonteCarloFollowedByQTTagging408Linear.cpp (include/mdmc.h qt_model 1) at its own
    size, N = 4096: the pump period (plasmaToQuantumTimestepRatio QT steps + one MD step per MD step)
    and the recorded period's tagged moments + 3 x 4001-bin velocity distributions.  The reference
    needs Armadillo (absent): no CPU baseline."""
    import tempfile
    from mdqtplasmasims_amd import mdmc
    tmp = tempfile.mkdtemp(prefix="qtt_bench_")
    e = mdmc.MonteCarloMD(qt_model=1, device=local, seed=3, saveDirectory=tmp + "/")
    e.init()
    ratio = int(e.const("plasmaToQuantumTimestepRatio"))
    e.qsteps(ratio)
    e.md_steps(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        e.qsteps(ratio)
        e.md_steps(1)
    pump_ms = (time.perf_counter() - t0) / steps * 1e3
    e.tag_qt()
    e.tagged_moments_qt()
    t0 = time.perf_counter()
    for _ in range(steps):
        e.tagged_moments_qt()
    kde_ms = (time.perf_counter() - t0) / steps * 1e3
    N = e.N
    e.close()
    return {"workload": "MonteCarloFollowedByQTTagging408Linear.cpp: N=4096, n=2, pump 62 QT steps per MD step",
            "N": N, "qsteps_per_md_step": ratio, "pump_ms_per_md_step": pump_ms,
            "particle_qsteps_per_s": N * ratio / (pump_ms * 1e-3),
            "tagged_moments_and_distribution_ms": kde_ms, "cpu_baseline": None}


# the headline line: the contract's keys, the roofline and CPU baseline in brief, one compact entry per
# secondary line; everything else (censuses, PMC blocks, tail notes, samples) is the detail line
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "comm_size", "steps", "warmup", "ms_per_step",
             "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "timed_region_s")
HEAD_CONFIG_KEYS = ("workload", "N", "md_steps", "qsteps_per_md_step", "particle_md_steps_per_s", "parallelism", "rng")
HEAD_ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "avg_launch_us",
                  "hbm_frac_8d", "traffic_frac", "compulsory_hbm_frac")
HEAD_CPU_KEYS = ("value", "unit", "cores", "kind", "sample")
LINE_KEYS = ("value", "unit", "N", "n_gpus", "ms_per_md_step", "force_breakdown_ms")
LINE_ROOF_KEYS = ("bound", "frac", "fp64_frac", "f32_frac", "algorithmic_equivalent_frac", "pairs_evaluated_frac",
                  "block_kernel_ms", "load_imbalance")


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _sig(x, n=5):
    """floats of a secondary line in brief to n significant digits (the detail line keeps them whole)"""
    if isinstance(x, float):
        return float(f"{x:.{n}g}")
    if isinstance(x, dict):
        return {k: _sig(v, n) for k, v in x.items()}
    if isinstance(x, list):
        return [_sig(v, n) for v in x]
    return x


def compact_secondary(name, v):
    """one secondary line in brief: value, unit, N, ms per MD step, roofline frac and bound, parity ok,
    the CPU baseline's value"""
    if isinstance(v, list):                         # pump_models
        return [compact_secondary(name, x) for x in v]
    if not isinstance(v, dict):
        return v
    if "lines" in v:                                # jobs_per_gpu
        return {"lines": [dict(_pick(x, ("jobs", "value", "unit", "ms_per_md_step"))) for x in v["lines"]]}
    c = _pick(v, LINE_KEYS)
    if name == "mcmd":
        c.update(_pick(v, ("mc_steps_per_s", "md_steps_per_s", "md_particle_steps_per_s", "main_estimate_s")))
        if isinstance(v.get("qt_tagging"), dict):
            c["qt_tagging_particle_qsteps_per_s"] = v["qt_tagging"].get("particle_qsteps_per_s")
    if "qt_model" in v:
        c["qt_model"] = v["qt_model"]
    r = v.get("roofline")
    if isinstance(r, dict):
        c["roofline"] = _pick(r, LINE_ROOF_KEYS)
        pm = r.get("pmc")
        if isinstance(pm, dict) and pm.get("status") == "ok" and "valu_busy_frac" in pm:
            c["roofline"]["valu_busy_frac"] = pm["valu_busy_frac"]   # (the committed PMC summary of this tree)
    p = v.get("parity")
    if isinstance(p, dict):
        c["parity_ok"] = p.get("ok", None)
    cb = v.get("cpu_baseline")
    if isinstance(cb, dict) and "value" in cb:
        c["cpu_baseline"] = cb["value"]
    elif isinstance(cb, dict) and "main_estimate_s" in cb:   # mcmd: the reference build's main() estimate
        c["cpu_baseline_main_estimate_s"] = cb["main_estimate_s"]
    ft = v.get("force_tail")
    if isinstance(ft, dict) and "bound_met" in ft:
        c["force_tail_bound_met"] = ft["bound_met"]
    ep = v.get("epotential")
    if isinstance(ep, dict):
        c["epot_ms"] = ep.get("wall_ms")
    return c


def compact_line(out):
    """the headline JSON line (<= LINE_MAX_BYTES): the secondary lines are dropped from the end, largest
    first, if it ever grows past the budget (they stay in the detail line)"""
    h = _pick(out, HEAD_KEYS)
    h["config"] = _pick(out.get("config", {}), HEAD_CONFIG_KEYS)
    h["roofline"] = _pick(out.get("roofline") or {}, HEAD_ROOF_KEYS)
    cb = out.get("cpu_baseline")
    h["cpu_baseline"] = _pick(cb, HEAD_CPU_KEYS) if isinstance(cb, dict) else None
    if isinstance(cb, dict) and isinstance(cb.get("single_thread"), dict):
        h["cpu_baseline"]["single_thread_value"] = cb["single_thread"].get("value")
    sec = {k: _sig(compact_secondary(k, v)) for k, v in out.items() if k not in HEAD_KEYS and k not in
           ("config", "roofline", "cpu_baseline", "secondary_errors", "run_s")}
    h["lines"] = sec
    if out.get("secondary_errors"):
        h["secondary_errors"] = {k: str(e)[:200] for k, e in out["secondary_errors"].items()}
    if "run_s" in out:
        h["run_s"] = out["run_s"]
    while len(json.dumps(h)) > LINE_MAX_BYTES and h["lines"]:
        big = max(h["lines"], key=lambda k: len(json.dumps(h["lines"][k])))
        h["lines"].pop(big)
        h.setdefault("lines_in_detail_only", []).append(big)
    return h


def emit(out, t_start=None):
    """the detail line (BENCH_DETAIL, stderr) then the headline line, last on stdout"""
    if t_start is not None:
        out["run_s"] = time.perf_counter() - t_start
    print("BENCH_DETAIL " + json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(compact_line(out)), flush=True)


class Watchdog:
    """Bounds the secondary line items: exceptions are recorded in the line, and if the deadline
    passes (e.g. a collective that never completes) rank 0 prints what it has and every rank exits."""

    def __init__(self, seconds, rank, out, t_start):
        import threading
        self.rank, self.out, self.lock, self.t_start = rank, out, threading.Lock(), t_start
        self.done = threading.Event()
        self.current = None
        self.t = threading.Thread(target=self._wait, args=(seconds,), daemon=True)
        self.t.start()

    def _wait(self, seconds):
        if self.done.wait(seconds):
            return
        with self.lock:
            if self.rank == 0:
                self.out.setdefault("secondary_errors", {})[self.current or "?"] = \
                    f"did not finish within {seconds:.0f} s (watchdog)"
                emit(self.out, self.t_start)
            sys.stdout.flush()
            os._exit(0)

    def run(self, name, fn):
        self.current = name
        try:
            res = fn()
        except Exception as e:                       # noqa: BLE001 - reported in the line
            res, err = None, f"{type(e).__name__}: {e}"
        else:
            err = None
        with self.lock:
            if self.rank == 0:
                if err is None:
                    self.out[name] = res
                else:
                    self.out.setdefault("secondary_errors", {})[name] = err

    def finish(self):
        self.done.set()


def replicas_line(local, cfg, counts=(2, 4, 8), steps=100):
    """The reference's production pattern is an array of independent jobs (exampleSlurmFile.slurm:3,
    job = 1..8).  Here k of them share ONE MI355X, each context on its own HIP stream, MD steps
    issued round-robin from one host thread: one system's latency-bound QT launch overlaps another's
    force launch.  value = sum over jobs of N x qsteps / wall.  A capacity figure for the
    job-array workload, not the single-system headline."""
    import mdqtplasmasims_amd as M
    params, qt, desc = CONFIGS[cfg]
    res = []
    for k in counts:
        sims = [M.Simulation(device=local, seed=12345 + j, job=j, qt_enabled=qt, **params).init()
                for j in range(1, k + 1)]
        ratio = int(sims[0].const("plasmaToQuantumTimestepRatio"))
        for _ in range(5):
            for x in sims:
                x.md_steps(1)
        for x in sims:
            x.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            for x in sims:
                x.md_steps(1)
        for x in sims:
            x.synchronize()
        el = time.perf_counter() - t0
        ntot = sum(x.N for x in sims)
        for x in sims:
            x.close()
        res.append({"jobs": k, "N_total": ntot, "md_steps": steps, "ms_per_md_step": el / steps * 1e3,
                    "value": ntot * ratio * steps / el, "unit": "particle-qsteps/s"})
    return {"workload": desc + ": k independent jobs (seed 12345+job) on one GPU, one stream each",
            "lines": res}


def end_to_end_line(local, cfg, md_steps, base=40, warm=True):
    """mdqt_run() (SpeedUp main() loop :1248-1383) with the reference cadence: output() every
    sampleFreq = 40 MD steps (energies, KDE velocity distributions, state populations files),
    writeConditions at the end, files written.  mdqt_run() starts with init() (newRun = 1), so the
    rate is differential: two runs to different tmax (base and base + md_steps MD steps), value = extra
    particle-qsteps (particle-MD-steps without QT) / extra wall: init() and the final writeConditions
    cancel, the MD steps and the outputs between remain.  Large configs (C5, N = 1M):
    md_steps = 40, one output() — its Epotential() on the force call's plan — per 40 MD steps."""
    import tempfile
    import mdqtplasmasims_amd as M
    params, qt, desc = CONFIGS[cfg]

    def one(steps):
        with tempfile.TemporaryDirectory() as d:
            sim = M.Simulation(device=local, seed=12346, job=1, qt_enabled=qt, tmax=steps * 0.002,
                               saveDirectory=d + "/", **params)    # one MD step = 0.002 (SpeedUp:79-85)
            t0 = time.perf_counter()
            sim.run()
            sim.synchronize()
            el = time.perf_counter() - t0
            res = dict(N=sim.N, q=sim.qstep_index, c0=sim.counters()["c0"], wall=el,
                       files=sum(len(fs) for _, _, fs in os.walk(d)))
            sim.close()
        return res

    if warm:
        one(base)                                        # warm-up (module load, first allocations)
    a, b = one(base), one(base + md_steps)
    el, dq = b["wall"] - a["wall"], b["q"] - a["q"]
    dmd = b["c0"] - a["c0"]
    res = {"workload": desc + f", mdqt_run() with output() every 40 MD steps (files written): "
                              f"run to {b['c0']} MD steps minus run to {a['c0']}",
           "N": b["N"], "md_steps": dmd, "qsteps": dq, "outputs": (b["c0"] + 1) // 40 - (a["c0"] + 1) // 40,
           "files_long_run": b["files"], "wall_s": el, "wall_s_long_run_incl_init": b["wall"],
           "ms_per_md_step": el / dmd * 1e3 if dmd else None}
    if qt:
        res.update(value=b["N"] * dq / el, unit="particle-qsteps/s")
    else:
        res.update(value=b["N"] * dmd / el, unit="particle-MD-steps/s")
    return res


# the large-N dominant kernel: its plain instance, or (C3, C5: the skip radius reaches the image
# boundary) the one with the one-axis per-pair image (mdqt_forces.hip launch_forces_n3b)
N3B_KERNELS = ("void mdqt::k_pairs_n3b<1, false, false, false>(mdqt::N3BArgs)",
               "void mdqt::k_pairs_n3b<1, false, false, true>(mdqt::N3BArgs)",
               # the paired-wave kernel (option force_n3b_pairs, round 6)
               "void mdqt::k_pairs_n3b_pw<1, false, false, false>(mdqt::N3BArgs)",
               "void mdqt::k_pairs_n3b_pw<1, false, false, true>(mdqt::N3BArgs)")
N3B_KERNEL = N3B_KERNELS[0]


def latest_large_pmc(cfg):
    """the newest committed PMC summary of a large line (profiles/r<round><letter>_<cfg>_pmc.json)"""
    d = os.path.join(ROOT, "profiles")
    fs = sorted(f for f in os.listdir(d) if f.endswith(f"_{cfg}_pmc.json") and f.startswith("r"))
    return os.path.join(d, fs[-1]) if fs else None


def large_roofline(cfg, census, f_avg, k_avg, N, world, imbalance=None, pairs=0):
    """Roofline of a large line's dominant kernel, k_pairs_n3b.  VALU is the roof (30 flop per
    distinct pair, ~0 B per pair after staging).  `frac` is the block kernel's own rate on the pairs it
    evaluates, time-weighted over its two precisions: 30 flop x
    the census's f64 lane-steps / (world x 78.6 TF) plus 30 flop x its f32 lane-steps (the ultra-far f32
    form, ufar32_uniform) / (world x 157.3 TF) — the time at the roofs — over the kernel's average
    duration from its own HIP dispatch timestamps (k_avg, the timed force calls); skipped tile pairs and
    sub-tile groups excluded.  fp64_frac / f32_frac are the two terms.  Beside it:
    algorithmic_equivalent_frac — all N(N-1)/2 pairs in the same time, what 8(d) defines — and
    pairs_evaluated_frac, the evaluated share; force_call_frac — all pairs over the whole forces() call
    (sort, plan, kernel, reduction, tail pass, collectives).  With a PMC summary of the same config
    measured on this tree's kernel sources (world 1): VALU / SALU / LDS instructions per evaluated
    pair, the VALU issue-slot fraction, and the kernel's duration from the kernel trace."""
    tot = N * (N - 1) / 2.0
    ev = sum(v[0] for k, v in census.items() if not k.startswith("skip"))
    ev32 = sum(v[0] for k, v in census.items() if k in F32_TIERS)     # lane-steps in f32 (packed) pair forms
    ev64 = ev - ev32
    # mixed precision: the f64 lane-steps against the fp64 roof, the f32 ones against
    # the fp32 roof; frac = the time both would take at their roofs / the kernel's time (time-weighted),
    # `peak` the matching mixed roof, so that achieved / peak = frac
    t64 = W_F_PER_PAIR * ev64 / (FP64_PEAK_TFS * world * 1e12)
    t32 = W_F_PER_PAIR * ev32 / (FP32_PEAK_TFS * world * 1e12)
    peak = W_F_PER_PAIR * ev / (t64 + t32) / 1e12 if ev else FP64_PEAK_TFS * world
    peak64 = FP64_PEAK_TFS * world
    t = k_avg if k_avg else f_avg
    roof = {"bound": "fp64+fp32" if ev32 else "fp64", "kernel": N3B_KERNELS[2 if pairs else 0], "unit": "TFLOP/s", "peak": peak,
            "achieved": W_F_PER_PAIR * ev / t / 1e12, "frac": (t64 + t32) / t,
            "fp64_pairs_frac": ev64 / ev if ev else None, "f32_pairs_frac": ev32 / ev if ev else None,
            "fp64_frac": t64 / t, "f32_frac": t32 / t,
            "roofs": {"fp64": peak64, "fp32": FP32_PEAK_TFS * world,
                      "note": "frac = fp64_frac + f32_frac: 30 flop x the f64 lane-steps / fp64 roof + 30 flop x the "
                              "f32 lane-steps (ufar32_uniform) / fp32 roof, over the kernel's time"},
            "algorithmic_equivalent_frac": W_F_PER_PAIR * tot / t / 1e12 / peak64,
            "pairs_evaluated_frac": ev / tot,
            "force_call_frac": W_F_PER_PAIR * tot / f_avg / 1e12 / peak64,
            "block_kernel_ms": k_avg * 1e3 if k_avg else None, "force_call_ms": f_avg * 1e3,
            "evaluated_lane_steps": ev,
            "time": "k_pairs_n3b's own dispatch timestamps (HIP events, every timed force call; max over ranks)"
                    if k_avg else "force() HIP events (no block-kernel timestamps)",
            "tiers": {k: {"lane_steps": v[0], "ion_pairs": v[1], "pairs_frac": v[1] / tot} for k, v in census.items()},
            "traffic": None, "pmc": None}
    if imbalance is not None:
        roof["load_imbalance"] = imbalance
    path = latest_large_pmc(cfg)
    if world != 1 or not path:
        return roof
    with open(path) as f:
        d = json.load(f)
    meta = d.get("_meta", {})
    p = {"file": os.path.relpath(path, ROOT), "measured_src_hash": meta.get("src_hash"),
         "src_hash": kernel_source_hash(), "workload": meta.get("workload")}
    # the instance this config ran (the one the summary has dispatches of)
    kname = max(N3B_KERNELS, key=lambda k: (d.get(k) or {}).get("dispatches", 0))
    e = d.get(kname)
    roof["kernel"] = kname
    if meta.get("src_hash") != p["src_hash"] or not e:
        roof["pmc"] = dict(p, status="stale: measured on other kernel sources" if e else "kernel not in the summary")
        return roof
    w = ev / 64.0                                   # wave-level pair steps
    cyc = e.get("GRBM_GUI_ACTIVE", 0) / 8.0          # the kernel's cycles (summed over the 8 XCDs)
    p.update(status="ok", dispatches=e.get("dispatches"),
             valu_per_evaluated_pair=e["SQ_INSTS_VALU"] / w, salu_per_evaluated_pair=e.get("SQ_INSTS_SALU", 0) / w,
             lds_per_evaluated_pair=e.get("SQ_INSTS_LDS", 0) / w,
             valu_issue_frac=e["SQ_INSTS_VALU"] * 4.0 / (1024.0 * cyc) if cyc else None)
    if cyc and "SQ_ACTIVE_INST_VALU" in e:
        # the hardware's VALU occupancy (rocprofv3's VALUBusy: quad-cycles summed over the SIMDs / (CUs x the
        # kernel's cycles)) — each instruction at its real cost (the quarter-rate v_rsq_f64, the f32
        # transcendentals), where valu_issue_frac prices every VALU instruction at 4 cycles
        p.update(valu_busy_frac=e["SQ_ACTIVE_INST_VALU"] / (256.0 * cyc),
                 valu_dual_issue_frac=e.get("SQ_ACTIVE_INST_VALU2", 0.0) / (256.0 * cyc),
                 trans_per_valu=(e.get("SQ_INSTS_VALU_TRANS_F64", 0.0) + e.get("SQ_INSTS_VALU_TRANS_F32", 0.0))
                 / e["SQ_INSTS_VALU"])
    if e.get("duration_us"):
        ks = e["duration_us"] * 1e-6
        p.update(kernel_us=e["duration_us"], clock_ghz=cyc / ks / 1e9 if cyc else None,
                 algorithmic_equivalent_frac_pmc=W_F_PER_PAIR * tot / ks / 1e12 / peak64,
                 evaluated_frac_pmc=(t64 + t32) / ks)
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:    # kB; FETCH x 2 per MI355X_MICROARCH.md (gfx950)
        roof["traffic"] = (2.0 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024.0
    roof["pmc"] = p
    return roof


def sharded_run(cfg, steps, rank, world, local, dist, barrier):
    """C5 (or C3/C4) as ONE system whose ions are sharded over the world: strong scaling."""
    import torch
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_unique_id
    params, qt, desc = CONFIGS[cfg]
    sim = M.Simulation(device=local, world_size=world, rank=rank, seed=12346, job=1, qt_enabled=qt, **params)
    if world > 1:
        obj = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        sim.comm_init(obj[0])
    comm_size = sim.comm_size()                    # ncclCommCount of the product's communicator
    if comm_size != world:
        raise RuntimeError(f"RCCL communicator has {comm_size} ranks, world {world}")
    t0 = time.perf_counter()
    sim.init()                                     # collective: Epot0 over all slabs
    t_init = time.perf_counter() - t0
    ratio = int(sim.const("plasmaToQuantumTimestepRatio"))
    # parity against a world-1 run (below); MDQT_BENCH_PARITY=1 runs the same check at world 1 (the
    # code path of the check on a one-GPU box: the comparison is then world 1 against itself)
    check = world > 1 or os.environ.get("MDQT_BENCH_PARITY") == "1"
    if check:
        sim.forces()                               # the first call's forces, this rank's slab
        F0 = sim.get_state()["F"]
    sim.md_steps(1)
    barrier()
    # kinds: force calls, fused substeps, and the force-call breakdown (bit 3: events between the stages)
    sim.enable_timing(1, kinds=1 | 2 | 8)
    t0 = time.perf_counter()
    sim.md_steps(steps)
    sim.synchronize()
    barrier()
    el = time.perf_counter() - t0
    kt = sim.kernel_times()
    bd = sim.force_breakdown()
    f_ms, nf, s_ms, ns = kt["force_ms"], kt["n_force"], kt["substep_ms"], kt["n_substep"]
    k_avg = kt["block_ms"] / kt["n_block"] * 1e-3 if kt["n_block"] else 0.0
    # Epotential() (SpeedUp:244-281; output() calls it every sampleFreq MD steps, :948) after the window:
    # two calls, wall and (world 1, blocks) the potential calls' block kernel — VERDICT r05 item 2
    sim.enable_timing(1, kinds=4)
    t1 = time.perf_counter()
    for _ in range(2):
        epot = sim.Epotential()
    sim.synchronize()
    epot_ms = (time.perf_counter() - t1) / 2 * 1e3
    pk = sim.kernel_times()
    pot_k_ms = pk["pot_block_ms"] / pk["n_pot_block"] if pk["n_pot_block"] else 0.0
    sim.enable_timing(False)
    bkeys = list(sim.BREAKDOWN_KEYS)
    tt = torch.tensor([el, k_avg, epot_ms, pot_k_ms] + [bd[k] for k in bkeys], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, k_avg, epot_ms, pot_k_ms = float(tt[0]), float(tt[1]), float(tt[2]), float(tt[3])
    breakdown = {k: float(tt[4 + i]) for i, k in enumerate(bkeys)} if bd["calls"] else None
    N = sim.N
    L = sim.const("L")
    rt, tail = sim.const("force_skip_radius"), sim.const("force_tail_bound")
    n3b_pairs = int(sim.const("force_n3b_pairs"))   # the paired-wave block kernel (k_pairs_n3b_pw) or the 8-wave one
    tmode, tmodel = int(sim.const("force_tail_mode")), sim.const("force_tail_model_bound")
    fixed, raw = sim.const("force_tail_fixed_tiles"), sim.const("force_tail_raw_bound")
    rm, mid = sim.const("force_mid_radius"), sim.const("force_mid_bound")
    rf, far = sim.const("force_far_radius"), sim.const("force_far_bound")
    rv, vfar = sim.const("force_vfar_radius"), sim.const("force_vfar_bound")
    ru, ufar = sim.const("force_ufar_radius"), sim.const("force_ufar_bound")
    ru32 = sim.const("force_ufar32_radius")
    tail_eps = 10.0 ** -12                          # force_tail_exp default
    fmode = int(sim.const("force_form_measured"))   # force_form_mode >= 1: the sums hold the forms' terms too
    fshare = fmode and int(sim.const("force_form_mode")) == 2
    err_eps = sim.const("force_error_eps")          # what they are held to (tail eps + 1e-13 per active tier)
    bound_met = bool((fmode and tail <= err_eps) or (not fmode and (rt >= L / 2 or (tmode == 1 and tail <= tail_eps)
                                                                    or tmode == 0)))
    census = None                                  # the block kernel's work by tile-pair class
    imbalance = None
    if int(sim.const("force_scheme")) == 3 and int(sim.const("force_sort")) == 1:
        census = sim.force_census()                # (this rank's block pairs: summed over the ranks)
        if world > 1:
            keys = list(census)
            ev_r = sum(v[0] for k, v in census.items() if not k.startswith("skip"))
            t = torch.tensor([x for k in keys for x in census[k]], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            v = t.tolist()
            census = {k: (v[2 * i], v[2 * i + 1]) for i, k in enumerate(keys)}
            # load balance: this rank's evaluated lane-steps, max over mean
            m = torch.tensor([ev_r], dtype=torch.float64, device="cuda")
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
            ev_t = sum(v[0] for k, v in census.items() if not k.startswith("skip"))
            imbalance = float(m[0]) / (ev_t / world) if ev_t else None
    parity = None
    if check:
        # the sharded result against a world-1 context built from the same inputs
        # (init() is deterministic), run on each rank's own GPU through the same MD steps: every
        # rank compares its slab — the first call's forces, then R and V after 1 + steps MD steps —
        # and the maxima over the ranks decide (mdqtplasmasims_amd.sharded.sharded_parity)
        from mdqtplasmasims_amd.sharded import sharded_parity
        st = sim.get_state()
        lo, hi = sim.slab_bounds()
        sim.close()
        ref = M.Simulation(device=local, world_size=1, rank=0, seed=12346, job=1, qt_enabled=qt, **params).init()
        ref.forces()
        rF0 = ref.get_state()["F"]
        ref.md_steps(1 + steps)
        rs = ref.get_state()
        ref.close()

        def all_max(vals):
            t = torch.tensor(vals, dtype=torch.float64, device="cuda")
            if world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return [float(x) for x in t.tolist()]

        parity = sharded_parity({"F0": F0, "R": st["R"], "V": st["V"]}, {"F0": rF0, "R": rs["R"], "V": rs["V"]},
                                lo, hi, L, all_max)
        parity.update(comm_size=comm_size, md_steps_compared=1 + steps,
                      reference="a world-1 context of the same init() on each rank's GPU; each rank's slab "
                                "compared, max over ranks")
        if not parity["ok"]:
            raise RuntimeError(f"sharded result differs from world 1: {json.dumps(parity)}")
    else:
        sim.close()
    unit_steps = ratio if qt else 1
    f_avg = f_ms / max(nf, 1) * 1e-3
    pairs = N * (N - 1) / 2.0
    force = {"avg_ms": f_avg * 1e3, "launches": nf, "pairs_per_s": pairs / f_avg if f_avg else None,
             "fp64_tflops": W_F_PER_PAIR * pairs / f_avg / 1e12 if f_avg else None,
             "fp64_frac": W_F_PER_PAIR * pairs / f_avg / 1e12 / FP64_PEAK_TFS if f_avg else None,
             "note": "this rank's forces() (sort, plan, block kernel, slot reduction, tail pass, reduce-scatter; "
                     "the position all-gather runs just before it, force_breakdown_ms.allgather); flops = 30 x "
                     "N(N-1)/2 (SURVEY 8d)"}
    if breakdown is not None:
        # the stages of the timed force calls (events between them on the context stream,
        # max over ranks per stage); stages_sum = sort_boxes + ... + reduce_scatter, against force.avg_ms
        st = sum(breakdown[k] for k in bkeys[1:7])
        breakdown["stages_sum"] = st
        breakdown["stages_sum_vs_force_call"] = st / (f_avg * 1e3) if f_avg else None
        force["breakdown_note"] = ("force_breakdown_ms: allgather = the ncclAllGather before each timed call; "
                                   "sort_boxes (Hilbert sort, tile/sub-tile boxes; the first sharded call's balance "
                                   "census), plan, block_kernel, slot_reduce, tail_pass (ncclAllReduce of the tail "
                                   "sums, k_tail_max, k_tail_fix), reduce_scatter: consecutive intervals of forces()")
    epotential = {"Epot": epot, "wall_ms": epot_ms, "block_kernel_ms": pot_k_ms or None,
                  "vs_force_call": epot_ms / (f_avg * 1e3) if f_avg else None,
                  "mode": ("the force call's plan (potential_plan 1): skips, sub-tile groups, error-bounded forms, "
                           "the enforced tail" if world == 1 and pot_k_ms else
                           "owner-computes rows, every pair to L/2" if world > 1 else "exact, every pair to L/2")}
    return {"workload": desc + ", one system sharded over all ranks (RCCL position all-gather; "
                           "Newton-3 block-pair forces reduce-scattered)",
            "N": N, "n_gpus": world, "comm_size": comm_size, "md_steps": steps, "ms_per_md_step": el / steps * 1e3,
            "value": N * unit_steps * steps / el,
            "unit": "particle-qsteps/s" if qt else "particle-MD-steps/s",
            "scaling": "strong", "init_s": t_init, "force": force, "force_breakdown_ms": breakdown,
            "epotential": epotential,
            "roofline": large_roofline(cfg, census, f_avg, k_avg, N, world, imbalance, n3b_pairs) if census and f_avg else None,
            "parity": parity if check else {"note": "world 1: this line is the reference the sharded runs are checked against"},
            "force_tail": {"skip_radius": rt, "half_box": L / 2, "bound": tail, "bound_met": bound_met,
                           "tail_mode": "measured+enforced" if tmode == 1 else "a priori",
                           "form_mode": ("measured+enforced, shared budget" if fshare else "measured+enforced") if fmode
                           else "a priori", "error_eps": err_eps,
                           "tail_model_bound": tmodel if tmode == 1 else None,
                           "tiles_over_eps_fixed": fixed, "largest_tile_sum_before_fix": raw,
                           "mid_radius": rm, "mid_bound": mid,
                           "far_radius": rf, "far_bound": far, "vfar_radius": rv, "vfar_bound": vfar,
                           "ufar_radius": ru, "ufar_bound": ufar, "ufar32_radius": ru32,
                           "note": "tile pairs >= skip_radius apart are skipped (tail_mode measured+enforced: every "
                                   "call sums per 16-ion sub-tile n g(sub-box distance) over the pairs it drops, tiles over "
                                   "1e-12 are recomputed exactly (tiles_over_eps_fixed), bound is the largest "
                                   "remaining sub-tile sum; a priori: (N - 1) g(skip_radius)); sub-tile groups >= mid_radius / "
                                   "far_radius / vfar_radius / ufar_radius apart take the mid / far / very-far / ultra-far pair "
                                   "forms; every ion's force is within bound + mid_bound + far_bound + vfar_bound + ufar_bound "
                                   "of the exact sum to L/2 (mdqt_engine.cpp tail_radius / far_radius_l; 0 = exact); "
                                   "form_mode measured+enforced (round 6): the tiers' radii from a density model, the sums "
                                   "also hold n g(gap) err_form(gap) of every sub-block evaluated in an error-bounded form, "
                                   "held to error_eps, and bound (their largest after the exact pass) is every ion's total "
                                   "(the *_bound entries are then the model's); shared budget (force_form_mode 2): where the tail skips "
                                   "nothing its unused 1e-12 is split among the active tiers, so error_eps is the same "
                                   "1.5e-12 per ion as where the tail is active. fp64 rates count all N(N-1)/2 pairs (SURVEY 8d)"},
            "substeps_ms_per_md_step": s_ms / max(ns, 1) if ns else None}


if __name__ == "__main__":
    main()
