"""The sharded Newton-3 block-pair force protocol (N > 65,536 on one or more GPUs),
checked on the CPU — no GPU needed:

  * ownership: the cyclic half shell of block distances, split over ranks by blocks
    [Plo, Phi) and over workgroups by runs of distances, evaluates every distinct tile pair exactly
    once, for world sizes 1-8 and even / odd block counts.  `n3b_plan` restates
    mdqt_engine.cpp:choose_segments and `n3b_tile_pairs` the loops of
    mdqt_forces.hip:k_pairs_n3b (the same arithmetic, so a change there must be mirrored here);
  * forces: a world-2 gloo group where each rank evaluates its tile pairs into a dense partial
    force array, the partials are summed across ranks (the reduce-scatter step; gloo all-reduce,
    then every rank keeps its slab) and compared with the oracle's full forces() within 1e-13.
Cross-world tolerance: the GPU path sums the rank partials in RCCL's (or, in-process, rank) order,
so results for different world sizes agree to rounding (measured 1e-16 relative, gate 1e-13), not
bit for bit; below 65,536 ions the owner-computes rows scheme is bit-identical across world sizes
(tests/test_gpu_parity.py::test_sharded_local_group_bit_identical).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def n3b_plan(N, world, rank, BW=8, target=65536, cuts=None):
    """mdqt_engine.cpp:choose_segments / n3b_set_range (Newton-3 blocks): tiles, blocks, half-shell
    distances, this rank's blocks (equal counts, or the cut points `cuts` of n3b_balance), runs of
    distances per block"""
    T = (N + 63) // 64
    NB = (T + BW - 1) // BW
    nd = NB // 2 + 1
    Plo = rank * NB // world if cuts is None else cuts[rank]
    Phi = (rank + 1) * NB // world if cuts is None else cuts[rank + 1]
    nblk = max(Phi - Plo, 1)
    R = min(nd, (target + nblk - 1) // nblk)
    runlen = (nd + R - 1) // R
    R = (nd + runlen - 1) // runlen
    return dict(T=T, NB=NB, nd=nd, Plo=Plo, Phi=Phi, R=R, runlen=runlen, BW=BW)


def n3b_tile_pairs(N, world, rank, BW=8, cuts=None):
    """(I, J, diag) of every tile pair rank `rank` evaluates: mdqt_forces.hip:k_pairs_n3b's loops
    over workgroups (block P, run), distances db of the run, J tiles of block Q = P + db, waves I"""
    p = n3b_plan(N, world, rank, BW, cuts=cuts)
    T, NB, nd = p["T"], p["NB"], p["nd"]
    out = []
    for wg in range((p["Phi"] - p["Plo"]) * p["R"]):
        P = p["Plo"] + wg // p["R"]
        run = wg % p["R"]
        d0, d1 = run * p["runlen"], min(nd, run * p["runlen"] + p["runlen"])
        for db in range(d0, d1):
            if NB % 2 == 0 and db == NB // 2 and P >= NB // 2:
                continue                                  # the other half covers it
            Q = (P + db) % NB
            for b in range(BW):
                J = Q * BW + b
                if J >= T:
                    break
                for q in range(BW):                       # waves: I = P * BW + q
                    I = P * BW + q
                    if I < T and (db > 0 or J >= I):
                        out.append((I, J, db == 0 and J == I))
    return out


def balance_cuts(w, world):
    """mdqt_engine.cpp:n3b_balance: cut points with each rank's prefix work nearest r / W of the total,
    at least one block per rank"""
    pre = np.concatenate([[0.0], np.cumsum(np.asarray(w, dtype=float))])
    NB, tot = len(w), pre[-1]
    cut = [0] * (world + 1)
    cut[world] = NB
    for r in range(1, world):
        t = tot * r / world
        k = int(np.searchsorted(pre, t, side="left"))
        if k > 0 and t - pre[k - 1] < pre[k] - t:
            k -= 1
        cut[r] = min(max(k, cut[r - 1] + 1), NB - (world - r))
    return cut


@pytest.mark.parametrize("N,BW", [(64 * 40 + 17, 2), (64 * 97 - 5, 4), (64 * 64, 16)])
def test_weighted_block_ranges_cover_every_tile_pair_once(N, BW):
    """the work-weighted block ranges (force_balance 1) are another partition of the blocks: every
    distinct tile pair still exactly once, for skewed work profiles and world sizes 2-8"""
    T = (N + 63) // 64
    NB = (T + BW - 1) // BW
    rng = np.random.default_rng(2)
    for prof in (rng.uniform(0.2, 1.8, NB), np.linspace(0.3, 1.7, NB), np.r_[np.full(NB // 2, 5.0), np.ones(NB - NB // 2)]):
        for world in range(2, min(8, NB) + 1):        # (n3b_balance keeps equal counts when NB < W)
            cuts = balance_cuts(prof, world)
            assert cuts[0] == 0 and cuts[-1] == NB and all(b > a for a, b in zip(cuts, cuts[1:]))
            seen = {}
            for rank in range(world):
                for I, J, diag in n3b_tile_pairs(N, world, rank, BW, cuts=cuts):
                    key = (min(I, J), max(I, J))
                    seen[key] = seen.get(key, 0) + 1
            assert len(seen) == T * (T + 1) // 2 and set(seen.values()) == {1}, (N, BW, world)
            per = [prof[cuts[r]:cuts[r + 1]].sum() for r in range(world)]
            # within one block's work of the ideal share
            assert max(per) <= prof.sum() / world + prof.max() + 1e-9


@pytest.mark.parametrize("N,BW", [(64 * 40 + 17, 2), (64 * 48, 3), (64 * 33 + 1, 4), (64 * 64, 16), (64 * 97 - 5, 4)])
def test_block_ownership_covers_every_tile_pair_once(N, BW):
    T = (N + 63) // 64
    for world in range(1, 9):
        seen = {}
        for rank in range(world):
            for I, J, diag in n3b_tile_pairs(N, world, rank, BW):
                key = (min(I, J), max(I, J))
                assert (I == J) == diag
                seen[key] = seen.get(key, 0) + 1
        assert len(seen) == T * (T + 1) // 2, (N, BW, world)
        assert set(seen.values()) == {1}, (N, BW, world)


def test_block_ownership_at_the_reference_sizes():
    """block level at C3 / C5 / N = 1M with the kernel's 16-tile blocks: every unordered block pair
    (and every block with itself) is owned by exactly one rank, world sizes 1-8"""
    for N in (99882, 249970, 1000258):
        for world in range(1, 9):
            seen = {}
            NB = None
            for rank in range(world):
                p = n3b_plan(N, world, rank)
                NB, nd = p["NB"], p["nd"]
                for P in range(p["Plo"], p["Phi"]):
                    for db in range(nd):
                        if NB % 2 == 0 and db == NB // 2 and P >= NB // 2:
                            continue
                        Q = (P + db) % NB
                        key = (min(P, Q), max(P, Q))
                        seen[key] = seen.get(key, 0) + 1
            assert len(seen) == NB * (NB + 1) // 2 and set(seen.values()) == {1}, (N, world)


def partial_forces(R, L, lDeb, pairs):
    """dense partial forces [3][N] of the given tile pairs: +f on the i side, -f on the j side, the
    reference's pair law (SpeedUp:213-230)"""
    N = R.shape[1]
    F = np.zeros((3, N))
    for I, J, diag in pairs:
        i0, i1 = I * 64, min(N, I * 64 + 64)
        j0, j1 = J * 64, min(N, J * 64 + 64)
        d = R[:, i0:i1, None] - R[:, None, j0:j1]
        d -= L * np.trunc(d / L + np.copysign(0.5, d))          # round half away from zero
        r = np.sqrt((d * d).sum(0))
        with np.errstate(divide="ignore", invalid="ignore"):
            ft = np.where((r > 0) & (r < L / 2), (1.0 / r + 1.0 / lDeb) * np.exp(-r / lDeb) / (r * r), 0.0)
        if diag:
            ft = np.triu(ft, 1)
        f = d * ft
        F[:, i0:i1] += f.sum(2)
        F[:, j0:j1] -= f.sum(1)
    return F


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
        from mdqtplasmasims_amd.engine import slab
        from oracle import oracle as O
        o = O.OracleSim(N0=3000, seed=77, rng_mode=1)
        L, lDeb = o.const("L"), o.const("lDeb")
        N = 3001
        R = np.random.default_rng(8).uniform(0, L, (3, N))
        BW = 2                                            # small blocks: many blocks at this N
        F = partial_forces(R, L, lDeb, n3b_tile_pairs(N, world, rank, BW))
        t = torch.from_numpy(F.copy())
        dist.all_reduce(t)                                # the reduce-scatter step (sum of partials)
        lo, hi, _ = slab(N, world, rank)
        mine = t.numpy()[:, lo:hi]
        G = O.forces_raw(R, L, lDeb)[:, lo:hi]
        q.put((rank, {"rel": float(np.abs(mine - G).max() / np.abs(G).max()), "slab": (lo, hi)}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, {"error": repr(e)}))


def test_block_partials_reduce_to_the_oracle_forces_gloo_world2(orc):
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
    for r, out in res.items():
        assert "error" not in out, out
        assert out["rel"] < 1e-13, out
    assert res[0]["slab"][1] == res[1]["slab"][0]


# ---------------------------------------------------------------------------------------------
# k_n3b_plan's pairing word (round 6): the lane-parallel form — each of lanes 0..BW-1 counts the tiles
# ahead of its own (strictly more work, or equal work and a lower tile) and writes its 3-bit field —
# against the serial stable insertion sort it replaced (mdqt_forces.hip k_n3b_plan)
# ---------------------------------------------------------------------------------------------
def _pairing_serial(row):
    BW = len(row)
    ord_ = list(range(BW))
    for u in range(1, BW):
        v = u
        while v > 0 and row[ord_[v]] > row[ord_[v - 1]]:
            ord_[v], ord_[v - 1] = ord_[v - 1], ord_[v]
            v -= 1
    pr = 0
    for k in range(BW // 2):
        pr |= (ord_[k] | ord_[BW - 1 - k] << 3) << (6 * k)
    return pr


def _pairing_lanes(row):
    BW = len(row)
    pr = 0
    for t in range(BW):
        rk = sum(1 for k in range(BW) if row[k] > row[t] or (row[k] == row[t] and k < t))
        pr |= (t << (6 * rk)) if rk < BW // 2 else (t << (3 + 6 * (BW - 1 - rk)))
    return pr


def test_plan_pairing_word_lane_parallel_matches_serial_sort():
    rng = np.random.default_rng(7)
    cases = [[0] * 8, list(range(8)), list(range(8))[::-1], [5, 5, 1, 1, 9, 9, 0, 0]]
    cases += [list(rng.integers(0, 4, 8)) for _ in range(2000)]          # many ties
    cases += [list(rng.integers(0, 1 << 20, 8)) for _ in range(2000)]
    for row in cases:
        assert _pairing_lanes(row) == _pairing_serial(row), row
