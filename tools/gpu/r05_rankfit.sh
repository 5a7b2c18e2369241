#!/bin/bash
# per-rank block-kernel times (forward and reverse order) and class censuses of in-process rank groups
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/r05c_rank.err
for c in c5 c3; do for w in 8 4; do
  timeout -k 10 300 python3 -u tools/rank_balance.py $c $w > gpurun_out/r05c_rank_${c}_w${w}.json 2>> gpurun_out/r05c_rank.err || { tail -5 gpurun_out/r05c_rank.err; exit 1; }
done; done
python3 - <<'PY'
import json, numpy as np
for c in ("c5", "c3"):
    for w in (8, 4):
        d = json.load(open(f"gpurun_out/r05c_rank_{c}_w{w}.json"))
        for k in ("equal", "weighted"):
            e = d[k]
            ev = np.array([sum(v for kk, v in cl.items() if not kk.startswith("skip")) for cl in e["census_lane_steps"]])
            f, r, m = (np.array(e[x]) for x in ("block_kernel_ms_forward", "block_kernel_ms_reverse", "block_kernel_ms"))
            print(c, w, k, "lane", np.round(ev / ev.mean(), 3).tolist(), "fwd", np.round(f / f.mean(), 3).tolist(),
                  "rev", np.round(r / r.mean(), 3).tolist(), "mean max/mean", round(m.max() / m.mean(), 4))
PY
