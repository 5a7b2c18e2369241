"""Real RCCL collectives through the product path: WORLD_SIZE ranks (torch.distributed.run, gloo
rendezvous), rank r on device r % device_count, one RCCL communicator (mdqt_comm_init: the position
all-gather before every force evaluation, the Newton-3 block partials' reduce-scatter).  Every rank
also runs the same system at world 1 and compares its slab.

On a one-GPU box RCCL refuses two ranks on one device (ncclCommInitRank: invalid usage, "Duplicate
GPU detected" — measured, round 2), so a real multi-rank collective needs a multi-GPU node; the
script then reports RCCL_ONE_GPU REFUSED instead of failing.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29533 tools/rccl_one_gpu.py [N0] [md_steps]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch.distributed as dist
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_unique_id
    N0 = int(sys.argv[1]) if len(sys.argv) > 1 else 70000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    kw = dict(N0=N0, seed=19, rng_mode=1)
    ref = M.Simulation(**kw).init()           # every rank: the same world-1 initial state
    st = ref.get_state()
    ndev = M.device_count()
    sim = M.Simulation(world_size=world, rank=rank, device=rank % ndev, **kw)
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    try:
        sim.comm_init(obj[0])
    except M.MdqtError as e:
        if rank == 0:
            print(f"RCCL_ONE_GPU REFUSED world={world} devices={ndev}: {e}")
        sim.close()
        ref.close()
        dist.destroy_process_group()
        return
    sim.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
    sim.allgather_positions()                 # RCCL all-gather
    sim.forces()                              # Newton-3 blocks: RCCL reduce-scatter of the partials
    ref.forces()
    lo, hi = sim.slab_bounds()
    G = ref.get_state()["F"]
    F = sim.get_state()["F"][:, lo:hi]
    errF = float(np.abs(F - G[:, lo:hi]).max() / np.abs(G).max())
    sim.md_steps(steps)                       # all-gather + reduce-scatter every MD step, QT on
    ref.md_steps(steps)
    sim.synchronize()
    a, b = sim.get_state(), ref.get_state()
    errR = float(np.abs(a["R"][:, lo:hi] - b["R"][:, lo:hi]).max())
    errV = float(np.abs(a["V"][:, lo:hi] - b["V"][:, lo:hi]).max() / np.abs(b["V"]).max())
    scheme = int(sim.const("force_scheme"))
    res = [None] * world
    dist.all_gather_object(res, (rank, lo, hi, errF, errR, errV, scheme))
    if rank == 0:
        for r in res:
            print(f"rank {r[0]} ions [{r[1]}, {r[2]}) scheme {r[6]}: forces vs world 1 max|dF|/max|F| = "
                  f"{r[3]:.3e}; after {steps} MD steps max|dR| = {r[4]:.3e}, max|dV|/max|V| = {r[5]:.3e}")
        ok = all(r[3] < 1e-13 and r[4] < 1e-10 and r[5] < 1e-10 for r in res)
        print("RCCL_ONE_GPU", "OK" if ok else "FAIL", f"world={world} N={ref.N}")
    dist.barrier()
    sim.close()
    ref.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
