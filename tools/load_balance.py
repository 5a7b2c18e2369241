"""Load balance of the sharded Newton-3 block kernel, measured on one GPU.

Rank r of W owns blocks [r NB / W, (r + 1) NB / W) (mdqt_engine.cpp plan sizing); its block kernel
does the evaluated lane-steps of those blocks' workgroups.  mdqt_force_block_work at world 1 gives
every block's evaluated lane-steps for the reference's init() positions (k_n3b_census, the block
kernel's own classification), so each partition's per-rank work follows; reported: max / mean over
the ranks for W = 2, 4, 8, with equal block counts and with the work-weighted ranges the engine takes
(mdqt_engine.cpp n3b_balance, option force_balance), at init() and after 3 MD steps.

    python tools/load_balance.py [c4 c5 c1m] > profiles/r05_load_balance.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import mdqtplasmasims_amd as M  # noqa: E402


def partition(work, W, cuts=None):
    NB = len(work)
    if cuts is None:
        cuts = [r * NB // W for r in range(W + 1)]
    return np.array([work[cuts[r]:cuts[r + 1]].sum() for r in range(W)])


def balance_cuts(w, W):
    """mdqt_engine.cpp:n3b_balance's cut points (tests/test_n3b_protocol.py restates the same)"""
    pre = np.concatenate([[0.0], np.cumsum(np.asarray(w, dtype=float))])
    NB, tot = len(w), pre[-1]
    cut = [0] * (W + 1)
    cut[W] = NB
    for r in range(1, W):
        t = tot * r / W
        k = int(np.searchsorted(pre, t, side="left"))
        if k > 0 and t - pre[k - 1] < pre[k] - t:
            k -= 1
        cut[r] = min(max(k, cut[r - 1] + 1), NB - (W - r))
    return cut


def main():
    cfgs = sys.argv[1:] or ["c4", "c5", "c1m"]
    out = {}
    for cfg in cfgs:
        params, qt, desc = bench.CONFIGS[cfg]
        t0 = time.perf_counter()
        sim = M.Simulation(device=0, seed=12346, job=1, qt_enabled=qt, **params).init()
        res = {"workload": desc, "N": sim.N, "blocks": int(sim.const("n3b_block_count"))}
        for tag, steps in (("init", 0), ("after_3_md_steps", 3)):
            if steps:
                sim.md_steps(steps)
            w = sim.force_block_work()
            cen = sim.force_census()
            ev = sum(v[0] for k, v in cen.items() if not k.startswith("skip"))
            assert abs(w.sum() - ev) <= 1e-9 * ev, (w.sum(), ev)     # the per-block sums are the census
            row = {"evaluated_lane_steps": ev, "block_min_over_mean": float(w.min() / w.mean()),
                   "block_max_over_mean": float(w.max() / w.mean())}
            for W in (2, 4, 8):
                per = partition(w, W)
                row[f"world{W}_max_over_mean"] = float(per.max() / per.mean())
                row[f"world{W}_min_over_mean"] = float(per.min() / per.mean())
                pw = partition(w, W, balance_cuts(w, W))      # force_balance 1 (the product default)
                row[f"world{W}_weighted_max_over_mean"] = float(pw.max() / pw.mean())
            res[tag] = row
        sim.close()
        res["seconds"] = time.perf_counter() - t0
        out[cfg] = res
        print(cfg, json.dumps(res), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
