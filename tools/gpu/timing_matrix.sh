#!/bin/bash
# how the HIP-event kernel times of the C2 line depend on the window and the sampling period
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A="--no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
for cfg in "20 5 0" "20 5 0" "200 20 0" "20 5 0"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --steps $1 --warmup $2 --timing-period $3 $A > gpurun_out/tm.log 2>&1 || { tail -3 gpurun_out/tm.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/tm.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print('steps $1 period $3', 'step', round(d['ms_per_step']*1e3,2), 'force', round(k['force_total']/k['force_launches']*1e3,2), k['force_launches'], 'qt', round(k['substeps_total']/k['substep_launches']*1e3,2), k['substep_launches'])"
done
