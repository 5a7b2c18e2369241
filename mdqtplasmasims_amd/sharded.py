"""Multi-GPU launcher for particle-sharded runs: one process per GPU.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m mdqtplasmasims_amd.sharded <job> --N0=1000000 --qt=0 [--tmax=...] [--md-steps=K]

Each rank owns the slab of ions [rank*S, min((rank+1)*S, N)) (libmdqt `mdqt_slab`, a pure function
of N and the world size).  Data-path collectives per MD step, issued inside libmdqt on the
context's stream over xGMI: the RCCL all-gather of the position slabs before every force
evaluation, and — with Newton-3 block pairs (N > 65,536: every sharded BASELINE config) — one
reduce-scatter of the ranks' dense partial forces (each rank evaluates its blocks' pairs for all
ions).  Output steps all-reduce scalars, the 3 x 2001 KDE bins and the per-ion file columns; rank 0
writes the reference's files.  torch.distributed (gloo) is used only for the rendezvous: rank 0
creates the RCCL unique id and broadcasts it.

World-size invariance: the quantum-jump stream is keyed by the GLOBAL ion id.  With the
owner-computes rows scheme (N <= 65,536, or force_scheme 1) force rows do not depend on the slab
(the j-segmentation is a function of N only), so 1/2/4/8-GPU runs are bit-identical
(tests/test_gpu_parity.py::test_sharded_local_group_bit_identical).  With Newton-3 block pairs
the rank partials are summed in the reduce-scatter's order, so results for different world sizes
agree to rounding, not bit for bit: forces within 1e-13 of world 1, two MD steps within 1e-12
(tests/test_gpu_large.py::test_sharded_newton3_blocks_above_64k_local_group,
tests/test_n3b_protocol.py for the block ownership and the partial reduction over gloo).
"""
from __future__ import annotations

import argparse
import os
import sys

from .engine import Simulation, comm_unique_id, slab


def dist_env():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def broadcast_uid(make_uid, rank: int) -> bytes:
    """rank 0 calls make_uid(); everybody receives its bytes (torch.distributed object broadcast)."""
    import torch.distributed as dist
    obj = [make_uid() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def check_partition(N: int, rank: int, world: int):
    """all ranks agree on the slab partition and it covers [0, N) exactly once."""
    import torch
    import torch.distributed as dist
    lo, hi, S = slab(N, world, rank)
    mine = torch.tensor([lo, hi, S], dtype=torch.int64)
    allb = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allb, mine)
    b = [tuple(int(x) for x in t) for t in allb]
    assert b[0][0] == 0 and b[-1][1] == N, b
    assert all(b[r][1] == b[r + 1][0] for r in range(world - 1)), b
    assert len({x[2] for x in b}) == 1, b
    return lo, hi, S


PARITY_TOL = 1e-12


def sharded_parity(mine: dict, ref: dict, lo: int, hi: int, L: float, all_max, tol: float = PARITY_TOL) -> dict:
    """A sharded run checked against a world-1 run of the same inputs (bench.py's sharded lines;
    SURVEY §8(e), reference scale-out exampleSlurmFile.slurm:3,16).

    mine / ref: "F0" (forces after the first forces() call), "R", "V" (after the same MD steps) as
    [3][N] arrays — of `mine` only this rank's slab [lo, hi) is read (a rank's copies of the other
    slabs are stale between all-gathers).  all_max(list of floats) -> their element-wise maximum over
    the ranks (torch.distributed all_reduce MAX: RCCL on the GPU box, gloo in the CPU test).
    Relative errors: forces by max|F|, positions by L, velocities by max|V| — every rank's slab, so
    one bad rank fails the check on all of them.  ok: max_rel_err <= tol (NaN fails)."""
    import numpy as np
    loc = []
    for k in ("F0", "R", "V"):
        a, b = np.asarray(mine[k])[:, lo:hi], np.asarray(ref[k])[:, lo:hi]
        if hi > lo:
            d = np.abs(a - b)
            loc += [float(d.max()) if np.all(np.isfinite(d)) else float("inf"), float(np.abs(b).max())]
        else:
            loc += [0.0, 0.0]
    dF, sF, dR, _, dV, sV = all_max(loc)
    rel = {"F0": dF / sF if sF > 0 else dF, "R": dR / L, "V": dV / sV if sV > 0 else dV}
    m = max(rel.values())
    return {"max_rel_err": m, "rel_err": rel, "tol": tol, "ok": bool(m <= tol)}


def create(params: dict, rank: int, world: int, local_rank: int) -> Simulation:
    """one rank's context with its RCCL communicator (collective over the world)."""
    sim = Simulation(world_size=world, rank=rank, device=local_rank, **params)
    if world > 1:
        sim.comm_init(broadcast_uid(comm_unique_id, rank))
    return sim


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("job", type=int)
    ap.add_argument("--md-steps", type=int, default=0, help="run K MD steps instead of the full time loop")
    args, rest = ap.parse_known_args(argv)
    params = {"job": args.job}
    for a in rest:
        if not a.startswith("--") or "=" not in a:
            ap.error(f"bad parameter {a}")
        k, v = a[2:].split("=", 1)
        k = {"qt": "qt_enabled"}.get(k, k)
        params[k] = v if k == "saveDirectory" else (float(v) if "." in v or "e" in v.lower() else int(v))
    params.setdefault("seed", 12345 + args.job)
    rank, world, local = dist_env()
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    sim = create(params, rank, world, local)
    if args.md_steps > 0:
        sim.init()
        sim.md_steps(args.md_steps)
        sim.synchronize()
        if rank == 0:
            print(f"N={sim.N} t={sim.t:.6f} md_steps={args.md_steps}")
    else:
        sim.run()
        if rank == 0:
            print(sim.N)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    sim.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
