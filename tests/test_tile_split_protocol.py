"""The Newton-3 tile kernel's workgroup table (one GPU, N <= 65,536; the C2 headline), checked on the
CPU — no GPU needed.  `tile_table` restates mdqt_engine.cpp:tile_split_count and ensure_aux's table
(the plain table, and the split table that runs the last round's whole tile pairs in halves or
quarters), `wg_work` restates mdqt_pairs.hpp:n3_tile's rotation steps and slot stores (the same
arithmetic, so a change there must be mirrored here).  Checked for C2 (56 tiles on 256 CUs) and a
range of tile and CU counts:

  * every distinct ion pair of every tile pair is evaluated exactly once (and no ion with itself);
  * no two workgroups store the same (slot, ion) — the extra slots of the split pairs' later parts
    hold disjoint tiles — and every slot entry an ion's force sums is written by exactly one
    workgroup or stays the zero of the table build;
  * the split table's last round (the workgroups after the first floor(W / CUs) rounds) holds only
    half-size (option 1) or quarter-size (option 2) work.
"""
import itertools

import numpy as np
import pytest


def split_count(nt, ncu, mode):
    """mdqt_engine.cpp:tile_split_count"""
    if not mode or nt < 2:
        return 0
    w0 = nt * (nt + 1) // 2
    if w0 <= ncu or w0 > 8 * ncu:
        return 0
    k = w0 % ncu - nt
    last = 4 * k + 2 * nt if mode == 2 else 2 * k + nt
    return k if (k > 0 and last <= ncu and 2 * k <= nt) else 0


def split_slots(k, mode):
    """mdqt_engine.cpp:split_slots"""
    return (4 if mode == 2 else 1) if k > 0 else 0


def tile_table(nt, ncu, mode):
    """ensure_aux's workgroup table: (I, J, log2 parts, part) per workgroup"""
    k = split_count(nt, ncu, mode)
    if k == 0:
        return [(I, J, 0, 0) for I in range(nt) for J in range(I + 1, nt)] + [(I, I, 0, 0) for I in range(nt)], 0

    def split(I, J):
        return J == I + 1 and I % 2 == 0 and I < 2 * k

    h = [(I, J, 0, 0) for I in range(nt) for J in range(I + 1, nt) if not split(I, J)]
    if mode == 2:
        h += [(2 * m, 2 * m + 1, 2, p) for p in range(4) for m in range(k)]
        h += [(I, I, 1, p) for p in range(2) for I in range(nt)]
    else:
        h += [(2 * m, 2 * m + 1, 1, 0) for m in range(k)]
        h += [(I, I, 0, 0) for I in range(nt)]
        h += [(2 * m, 2 * m + 1, 1, 1) for m in range(k)]
    return h, k


_Q, _L = np.meshgrid(np.arange(4), np.arange(64), indexing="ij")


def wg_work(I, J, pl, part, nt):
    """n3_tile: the (ion i, ion j) pairs one workgroup evaluates (4 waves x 64 lanes; lane l of wave q
    at rotation step t meets J-ion (l + 16 q + t) mod 64 off the diagonal, (l + 1 + 8 q + t) mod 64 on
    it, the distance-32 step only for lanes < 32) as two arrays, and the (slot, ion) entries it stores"""
    diag = I == J
    ii, jj = [], []
    if not diag:
        n = 16 >> pl
        steps = range(part * n, part * n + n)
    else:
        steps = range(4 * part, 4 * part + 4) if pl else range(8)
    for t in steps:
        if not diag:
            jl = (_L + 16 * _Q + t) % 64
            keep = np.ones_like(jl, dtype=bool)
        else:
            d = 1 + 8 * _Q + t
            jl = (_L + d) % 64
            keep = ~((d == 32) & (_L >= 32))        # weight 0: lane distance 32 once per pair
        ii.append((64 * I + _L)[keep])
        jj.append((64 * J + jl)[keep])
    xs = -1 if part == 0 else (nt + 3 if diag else nt + part - 1)
    rows_i = xs if xs >= 0 else (I if diag else J)
    stores = [(rows_i, 64 * I + l) for l in range(64)]
    if not diag:
        rows_j = xs if xs >= 0 else I
        stores += [(rows_j, 64 * J + l) for l in range(64)]
    return np.concatenate(ii), np.concatenate(jj), stores


@pytest.mark.parametrize("nt,ncu,mode", [(56, 256, 1), (56, 256, 2), (56, 256, 0), (55, 256, 1), (40, 128, 1),
                                         (40, 128, 2), (30, 104, 1), (23, 64, 2), (64, 256, 1)])
def test_tile_table_covers_every_pair_once_and_stores_once(nt, ncu, mode):
    table, k = tile_table(nt, ncu, mode)
    nslots = nt + split_slots(k, mode)
    N = 64 * nt
    count = np.zeros(N * N, dtype=np.int32)
    stored = {}
    for w, (I, J, pl, part) in enumerate(table):
        a, b, stores = wg_work(I, J, pl, part, nt)
        assert not np.any(a == b)
        np.add.at(count, np.minimum(a, b) * N + np.maximum(a, b), 1)
        for st in stores:
            assert 0 <= st[0] < nslots
            assert st not in stored, (st, stored[st], w)
            stored[st] = w
    upper = np.triu(np.ones((N, N), dtype=bool), 1).ravel()
    assert np.all(count[upper] == 1) and not count[~upper].any()   # every distinct pair once, nothing else
    # every ion's slots: the ntiles plain slots are written for every ion (one tile pair with each tile)
    for ion in range(64 * nt):
        for slot in range(nt):
            assert (slot, ion) in stored
    if k:
        w0 = nt * (nt + 1) // 2
        first = (w0 // ncu) * ncu                    # workgroups of the full rounds
        assert len(table) - first == (4 * k + 2 * nt if mode == 2 else 2 * k + nt)
        for I, J, pl, part in table[first:]:         # the last round: half / quarter-size work only
            size = (0.5 if I == J else 1.0) / (1 << pl)
            assert size <= (0.25 if mode == 2 else 0.5)


def test_c2_split_counts():
    """C2 (N = 3,573: 56 tiles) on MI355X's 256 CUs: 1,596 workgroups, 60 past six rounds, 56 of them
    diagonal — 4 tile pairs split; 55 tiles (N0 = 3500 at other seeds): 1,540, nothing to split"""
    assert split_count(56, 256, 1) == 4 and split_count(56, 256, 2) == 4
    assert len(tile_table(56, 256, 1)[0]) == 1600 and len(tile_table(56, 256, 2)[0]) == 1536 + 128
    assert split_count(55, 256, 1) == 0
    assert all(split_count(nt, ncu, m) == 0 for nt, ncu, m in itertools.product([1, 2, 8], [256], [1, 2]))
