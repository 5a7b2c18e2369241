#!/bin/bash
# the timed window's fixed cost: 20- and 200-step windows with the one event-timed launch of the
# dominant kernel in the middle, first or last MD step of the window
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A="--no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
for rep in 1 2 3; do
for tl in mid first last; do
for st in 20 200; do
  timeout -k 10 200 python3 bench.py --steps $st --warmup 5 --timed-launch $tl $A > gpurun_out/win_${tl}_$st.log 2>&1 || { echo "$tl $st failed"; tail -5 gpurun_out/win_${tl}_$st.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/win_${tl}_$st.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print('$tl steps $st', round(d['ms_per_step']*1e3,2), 'qt', round(k['substeps_total']/k['substep_launches']*1e3,2), 'n', k['substep_launches'])"
done; done; done
