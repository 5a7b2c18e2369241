#!/usr/bin/env python3
"""CPU model of the Newton-3 block kernel's work in spatial order, and of finer culling inside a
tile pair (DESIGN.md §3 "Forces").

Positions uniform in the box (init() is), ordered by the engine's 30-bit Hilbert key
(mdqt_sort.hip k_curve_keys, restated), tiles of 64 and sub-tiles of 16 ions with minimum-image
boxes as k_tile_boxes computes them.  For a random sample of tile pairs (I < J):

  * now       the kernel: a tile pair is skipped when its boxes are >= r_s apart (r_s = the skip
              radius: L/2, or r_t < L/2 with the tail), else all 64 rotation steps run;
  * diag      16-ion sub-blocks, steps grouped by the 4 cyclic sub-block diagonals (lane group a
              meets J sub-tile (a + d) mod 4 for 16 steps): a diagonal runs iff one of its 4
              sub-blocks has sub-boxes < r_s apart;
  * matching  the same with the fewest groups: a 4 x 4 bipartite graph of active sub-blocks is
              covered by max-degree perfect matchings (Konig), 16 steps each;
  * step      per rotation step of the present kernel: a step runs iff one of its 64 pairs has
              sub-boxes < r_s apart (the measured-and-dropped per-step ballot).
Prints the lane-steps of each scheme per distinct pair and the fraction of pairs inside L/2.

    python tools/subtile_cull_model.py [C3|C5|C4|1M|C2] [samples]
"""
import sys

import numpy as np

CFG = {  # N, L, r_s (the skip radius the engine uses: L/2, or r_t from the tail model)
    "C2": (3573, 24.474785, None),
    "C3": (99882, 74.822038, None),
    "C5": (249970, 101.549129, None),
    "C4": (1000258, 161.199195, 68.07),
    "1M": (1000258, 161.199195, 62.03),
}


def hilbert_keys(R, L):
    q = np.clip((R * (1024.0 / L)).astype(np.int64), 0, 1023).astype(np.uint32)
    X = [q[0].copy(), q[1].copy(), q[2].copy()]
    Q = np.uint32(1 << 9)
    while Q > 1:
        P = np.uint32(Q - 1)
        m0 = (X[0] & Q) != 0
        X[0] = np.where(m0, X[0] ^ P, X[0])
        for i in (1, 2):
            mi = (X[i] & Q) != 0
            t = (X[0] ^ X[i]) & P
            X[0] = np.where(mi, X[0] ^ P, X[0] ^ t)
            X[i] = np.where(mi, X[i], X[i] ^ t)
        Q = np.uint32(Q >> 1)
    X[1] ^= X[0]
    X[2] ^= X[1]
    t = np.zeros_like(X[0])
    Q = np.uint32(1 << 9)
    while Q > 1:
        t = np.where((X[2] & Q) != 0, t ^ np.uint32(Q - 1), t)
        Q = np.uint32(Q >> 1)
    X = [x ^ t for x in X]

    def spread(x):
        x = x.astype(np.uint64) & 0x3FF
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        x = (x | (x << 2)) & 0x09249249
        return x
    return spread(X[2]) | (spread(X[1]) << 1) | (spread(X[0]) << 2)


def boxes(Rs, n, L):
    """center, half extent of groups of n consecutive ions (minimum image from the first one)"""
    G = Rs.shape[1] // n
    X = Rs[:, : G * n].reshape(3, G, n)
    d = X - X[:, :, :1]
    d -= L * np.rint(d / L)
    lo, hi = d.min(axis=2), d.max(axis=2)
    return X[:, :, 0] + 0.5 * (lo + hi), 0.5 * (hi - lo)


def gap2(ca, ha, cb, hb, L):
    d = ca - cb
    d -= L * np.rint(d / L)
    g = np.abs(d) - (ha + hb)
    return (np.where(g > 0, g, 0.0) ** 2).sum(axis=0)


def matchings(mask):
    """groups of 16 steps for an active 4x4 sub-block mask: the max degree (Konig)"""
    return np.maximum(mask.sum(axis=-1).max(axis=-1), mask.sum(axis=-2).max(axis=-1))


def main(cfg="C5", samples=20000, seed=1):
    N, L, rs = CFG[cfg]
    rs = L / 2 if rs is None else rs
    rng = np.random.default_rng(seed)
    R = rng.uniform(0, L, (3, N))
    Rs = R[:, np.argsort(hilbert_keys(R, L), kind="stable")]
    T = N // 64                                    # whole tiles only (the model ignores the ragged one)
    Rs = Rs[:, : T * 64]
    c64, h64 = boxes(Rs, 64, L)
    c16, h16 = boxes(Rs, 16, L)
    I = rng.integers(0, T, samples)
    J = rng.integers(0, T, samples)
    keep = I != J
    I, J = I[keep], J[keep]
    n = len(I)
    g = gap2(c64[:, I], h64[:, I], c64[:, J], h64[:, J], L)
    run = g < rs * rs                              # the tile pair is evaluated
    # sub-block gaps [n, 4, 4]
    a = 4 * I[:, None] + np.arange(4)[None, :]
    b = 4 * J[:, None] + np.arange(4)[None, :]
    sg = gap2(c16[:, a][:, :, :, None], h16[:, a][:, :, :, None], c16[:, b][:, :, None, :], h16[:, b][:, :, None, :], L)
    act = (sg < rs * rs) & run[:, None, None]
    diag = np.zeros(n)
    for d in range(4):
        diag += act[:, np.arange(4), (np.arange(4) + d) % 4].any(axis=1)
    match = matchings(act)
    # (round 6) 8-ion quadrants: group d's 16 steps as two 8-step halves, half h covering the quadrant
    # pairs (I half e, J half (e + h) mod 2) of each of the 4 lane rows; a half runs iff one of its 8
    # quadrant pairs has 8-ion boxes < r_s apart
    c8, h8 = boxes(Rs, 8, L)
    a8 = 8 * I[:, None] + np.arange(8)[None, :]
    b8 = 8 * J[:, None] + np.arange(8)[None, :]
    q8 = gap2(c8[:, a8][:, :, :, None], h8[:, a8][:, :, :, None], c8[:, b8][:, :, None, :], h8[:, b8][:, :, None, :], L)
    qact = (q8 < rs * rs) & run[:, None, None]        # [n, 8, 8]: I eighth 2a + e, J eighth 2b + f
    quad = np.zeros(n)
    for d in range(4):
        for h in range(2):
            on = np.zeros(n, dtype=bool)
            for a_ in range(4):
                b_ = (a_ + d) % 4
                for e in range(2):
                    on |= qact[:, 2 * a_ + e, 2 * b_ + (e + h) % 2]
            quad += on
    # per rotation step s of the present kernel: lane l (sub-tile l // 16) meets J index (l + s) % 64
    l = np.arange(64)
    steps = np.zeros(n)
    for s in range(64):
        steps += act[:, l // 16, ((l + s) % 64) // 16].any(axis=1)
    # useful pairs: inside L/2 (exact, on a sub-sample of the evaluated tile pairs)
    idx = np.nonzero(run)[0][:2000]
    inside = 0
    for k in idx:
        x = Rs[:, I[k] * 64:(I[k] + 1) * 64][:, :, None] - Rs[:, J[k] * 64:(J[k] + 1) * 64][:, None, :]
        x -= L * np.rint(x / L)
        inside += ((x ** 2).sum(axis=0) < (L / 2) ** 2).sum()
    frac_in = inside / (len(idx) * 4096) if len(idx) else 0.0
    tot = n * 4096.0
    print(f"{cfg}: N={N} L={L:.3f} r_s={rs:.3f}; {n} tile pairs sampled; evaluated tile pairs {run.mean():.3f}")
    print(f"  lane-steps per pair: now {run.sum() * 4096 / tot:.3f}, per-step ballot {steps.sum() * 64 / tot:.3f}, "
          f"cyclic diagonals {diag.sum() * 1024 / tot:.3f}, matchings {match.sum() * 1024 / tot:.3f}, "
          f"8-ion quadrant halves {quad.sum() * 512 / tot:.3f}")
    print(f"  pairs inside L/2 among the evaluated tile pairs: {frac_in:.3f} "
          f"(all pairs inside L/2: {np.pi / 6:.3f}); inside r_s: of all pairs "
          f"{4 * np.pi / 3 * rs ** 3 / L ** 3:.3f}")
    hist = np.bincount(match[run].astype(int), minlength=5) / max(run.sum(), 1)
    print(f"  evaluated tile pairs by matchings needed (0..4): {np.round(hist, 3).tolist()}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "C5", int(sys.argv[2]) if len(sys.argv) > 2 else 20000)
