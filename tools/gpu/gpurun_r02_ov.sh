#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
for ov in 1 0 1; do
for st in "200 20" "20 5"; do
set -- $st
timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --overlap $ov $A > gpurun_out/bench_ov.log 2>&1 || { tail -5 gpurun_out/bench_ov.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_ov.log').read().strip().splitlines()[-1]); print('overlap $ov steps $1', round(d['value']/1e9,4), round(d['ms_per_step']*1e3,2), d['config']['kernel_ms'])"
done
done
