#!/bin/bash
# bench large lines (C5 sharded path, N = 1M) alternating product / variants, force time per call
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A="--steps 3 --warmup 1 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line --md-only-config none"
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  timeout -k 10 400 env $lib python3 bench.py $A > gpurun_out/lab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/lab_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lab_$v.log').read().strip().splitlines()[-1])
print('$v', *[(k, round(d[k]['ms_per_md_step'], 2), round(d[k]['force']['avg_ms'], 2)) for k in ('sharded', 'sharded_1m') if k in d])"
done
