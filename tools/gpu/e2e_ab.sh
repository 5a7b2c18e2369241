#!/bin/bash
# A/B of the end-to-end (reference cadence, output() every 40 MD steps) line: base vs expt/<name>
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A="--steps 20 --warmup 5 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-replicas-line"
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  timeout -k 10 300 env $lib python3 bench.py $A > gpurun_out/e2e_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/e2e_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/e2e_$v.log').read().strip().splitlines()[-1]); e=d['end_to_end']; print('$v', 'e2e', round(e['value']/1e9,3), 'us/MDstep', round(e['wall_s']/e['md_steps']*1e6,2), 'headline', round(d['value']/1e9,3))"
done
