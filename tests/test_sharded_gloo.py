"""World-size-2 CPU tests (gloo) of the sharded multi-GPU protocol.

What runs here without a GPU:
  - the launcher's rendezvous (mdqtplasmasims_amd.sharded: unique-id broadcast, partition check)
    over a real 2-process gloo group, with libmdqt's own slab function;
  - the protocol itself — all-gather the position slabs, owner-computes force rows over all j,
    substeps of the owned slab with the quantum-jump stream keyed by GLOBAL ion id — executed
    with the oracle as the per-rank compute engine (test infrastructure), and checked bit for bit
    against a single-process run: partition invariance of the algorithm the GPU path shards.
The GPU side of the same protocol is covered by tests/test_gpu_parity.py (in-process rank group
on one MI355X, bitwise against world_size 1) and by bench.py's sharded check on the 8-GPU node.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from mdqtplasmasims_amd import sharded
        from mdqtplasmasims_amd.engine import slab
        from oracle import oracle as O

        out = {}
        # 1. rendezvous: every rank gets rank 0's id
        uid = sharded.broadcast_uid(lambda: bytes(range(128)), rank)
        out["uid_ok"] = uid == bytes(range(128))
        # 2. partition agreement for a few sizes
        for N in (0, 1, 63, 3573, 100000, 1000000):
            sharded.check_partition(N, rank, world)
        # 3. the sharded protocol with the oracle as compute engine
        kw = dict(N0=300, seed=4242, rng_mode=1)
        o = O.OracleSim(**kw).init()
        N = o.N
        L, lDeb = o.const("L"), o.const("lDeb")
        ratio = int(o.const("plasmaToQuantumTimestepRatio"))
        lo, hi, S = slab(N, world, rank)
        F0 = None
        for _ in range(3):
            st = o.get_state()
            buf = torch.zeros(world, 3, S, dtype=torch.float64)
            buf[rank, :, : hi - lo] = torch.from_numpy(st["R"][:, lo:hi])
            dist.all_gather_into_tensor(buf.view(-1), buf[rank].reshape(-1).clone())
            R = np.concatenate([buf[w].numpy() for w in range(world)], axis=1)[:, :N]
            o.set_state(R, st["V"], st["psi"], st["tPart"], st["t"])
            F = O.forces_rows(R, lo, hi, L, lDeb)
            F0 = F if F0 is None else F0
            o.set_forces(F)
            o.substeps(ratio)
        st = o.get_state()
        ref = O.OracleSim(**kw).init()
        rF0 = O.forces_raw(ref.get_state()["R"], L, lDeb)
        ref.md_steps(3)
        rs = ref.get_state()
        # 4. bench.py's sharded parity check (sharded.sharded_parity): each rank's slab against the
        # world-1 run, maxima over the ranks by all_reduce MAX; then rank 1's slab perturbed by 1e-9
        # of max|V| — every rank, rank 0 included, must see the failure
        def all_max(vals):
            t = torch.tensor(vals, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.tolist()
        mine = {"F0": F0, "R": st["R"], "V": st["V"]}
        refd = {"F0": rF0, "R": rs["R"], "V": rs["V"]}
        out["parity"] = sharded.sharded_parity(mine, refd, lo, hi, L, all_max)
        bad = dict(mine, V=st["V"].copy())
        if rank == 1:
            bad["V"][1, lo] += 1e-9 * np.abs(rs["V"]).max()
        out["parity_bad"] = sharded.sharded_parity(bad, refd, lo, hi, L, all_max)
        out["bitwise"] = all(np.array_equal(st[k][..., lo:hi] if k in ("R", "V") else st[k][lo:hi],
                                            rs[k][..., lo:hi] if k in ("R", "V") else rs[k][lo:hi])
                             for k in ("R", "V", "psi", "tPart"))
        out["t"] = (st["t"], rs["t"])
        out["slab"] = (lo, hi)
        q.put((rank, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, {"error": repr(e)}))


@pytest.fixture(scope="module")
def results(orc):
    from mdqtplasmasims_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from mdqtplasmasims_amd.build import build
        build(quiet=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return res


def test_no_errors(results):
    for r, out in results.items():
        assert "error" not in out, out


def test_uid_broadcast(results):
    assert all(out["uid_ok"] for out in results.values())


def test_slabs_cover_all_ions(results):
    lo0, hi0 = results[0]["slab"]
    lo1, hi1 = results[1]["slab"]
    assert lo0 == 0 and hi0 == lo1 and hi1 > lo1


def test_sharded_protocol_partition_invariant(results):
    for out in results.values():
        assert out["bitwise"]
        assert out["t"][0] == out["t"][1]


def test_sharded_parity_check(results):
    """bench.py's check of a sharded line against world 1: passes on the partition-invariant run
    (first forces, then R and V after 3 MD steps: bit for bit, so 0), and a 1e-9 error confined
    to rank 1's slab fails the check on both ranks"""
    for out in results.values():
        p, b = out["parity"], out["parity_bad"]
        assert p["ok"] and p["max_rel_err"] <= 1e-15, p
        assert not b["ok"] and 5e-10 < b["rel_err"]["V"] < 2e-9, b
        assert b["rel_err"]["F0"] == p["rel_err"]["F0"] and b["rel_err"]["R"] == p["rel_err"]["R"]
