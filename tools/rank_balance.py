"""Per-rank block-kernel time of a sharded force call, measured on one GPU: a world-W
in-process rank group whose ranks' force calls run one at a time (each synchronised), so each rank's
k_pairs_n3b runs alone on the MI355X; its own HIP dispatch timestamps give the rank's kernel time.
Equal block counts (force_balance 0) against the work-weighted ranges (1); forces checked against
world 1 (1e-13).

    python tools/rank_balance.py [cfg] [W]       (cfg c5 or c3; default c5 8)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main(cfg="c5", W=8):
    import mdqtplasmasims_amd as M
    from mdqtplasmasims_amd.engine import comm_init_local
    params, qt, desc = bench.CONFIGS[cfg]
    kw = dict(seed=12346, job=1, qt_enabled=qt, **params)
    ref = M.Simulation(**kw).init()
    st = ref.get_state()
    ref.forces()
    G = ref.get_state()["F"]
    ref.close()
    out = {"workload": desc, "world": W}
    for bal in (0, 1):
        sims = [M.Simulation(world_size=W, rank=r, **kw) for r in range(W)]
        for s in sims:
            s.set_state(st["R"], st["V"], st["psi"], st["tPart"], st["t"])
            s.set_option("force_balance", bal)
        comm_init_local(sims)
        for s in sims:
            s.allgather_positions()
        for s in sims:                                  # warm: the balance census, allocations
            s.forces()
            s.synchronize()
        for s in sims:
            s.get_state()
        for s in sims:
            s.allgather_positions()
        ev = []
        # each rank's call alone on the GPU, in rank order and then in reverse order (a drift of the
        # clock over the sequence shows as a trend in rank order; the mean of both passes cancels it)
        passes = []
        for order in (list(range(W)), list(range(W - 1, -1, -1))):
            t = [0.0] * W
            for _ in range(3):
                for r in order:
                    s = sims[r]
                    s.enable_timing(1, kinds=1)
                    s.forces()
                    s.synchronize()
                    kt = s.kernel_times()
                    s.enable_timing(0)
                    t[r] += kt["block_ms"] / max(kt["n_block"], 1) / 3
                for s in sims:                          # (the deferred reduce, then positions again)
                    s.get_state()
                for s in sims:
                    s.allgather_positions()
            passes.append(t)
        ms = [(a + b) / 2 for a, b in zip(*passes)]
        for s in sims:
            s.forces()
        worst = 0.0
        for s in sims:
            lo, hi = s.slab_bounds()
            worst = max(worst, np.abs(s.get_state()["F"][:, lo:hi] - G[:, lo:hi]).max() / np.abs(G).max())
        cls = []
        for s in sims:
            c = s.force_census()
            ev.append(sum(v[0] for k, v in c.items() if not k.startswith("skip")))
            cls.append({k: v[0] for k, v in c.items()})
        ranges = [(int(s.const("n3b_block_lo")), int(s.const("n3b_block_hi"))) for s in sims]
        ratio = sims[0].const("force_balance_ratio")
        for s in sims:
            s.close()
        ms, ev = np.array(ms), np.array(ev)
        out["weighted" if bal else "equal"] = {
            "block_ranges": ranges, "block_kernel_ms": ms.round(4).tolist(),
            "block_kernel_ms_forward": np.round(passes[0], 4).tolist(), "block_kernel_ms_reverse": np.round(passes[1], 4).tolist(),
            "kernel_max_over_mean": float(ms.max() / ms.mean()), "lane_steps_max_over_mean": float(ev.max() / ev.mean()),
            "engine_census_ratio": ratio, "max_rel_err_vs_world1": worst, "census_lane_steps": cls}
        brief = {k: v for k, v in out["weighted" if bal else "equal"].items() if k != "census_lane_steps"}
        print(cfg, "world", W, "balance", bal, json.dumps(brief), file=sys.stderr, flush=True)
        assert worst < 1e-13
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c5", int(sys.argv[2]) if len(sys.argv) > 2 else 8)
