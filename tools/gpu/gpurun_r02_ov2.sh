#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--steps 200 --warmup 20 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
run() {
  timeout -k 10 200 env $1 python3 bench.py $A --overlap $2 > gpurun_out/bench_ov.log 2>&1 || { tail -5 gpurun_out/bench_ov.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ov.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print('$1 ov=$2', round(d['value']/1e9,4), round(d['ms_per_step']*1e3,2), round(k['force_total']/k['force_launches']*1e3,1), round(k['substeps_total']/k['substep_launches']*1e3,1))"
}
run MDQT_OVL_SLEEP=2 0
run MDQT_OVL_MODE=1 1
run MDQT_OVL_SLEEP=16 1
run MDQT_OVL_SLEEP=64 1
