#!/bin/bash
# large-N tests on the product library, then the bench's large lines for the product and the given
# expt variants, alternating: bash tools/gpu/r03_large_ab.sh variant ...
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/r03_large.sh || exit $?
A="--steps 3 --warmup 1 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line --md-only-config none"
for v in "$@" base; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  timeout -k 10 400 env $lib python3 bench.py $A > gpurun_out/lab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/lab_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lab_$v.log').read().strip().splitlines()[-1])
print('$v', *[(k, round(d[k]['ms_per_md_step'], 2)) for k in ('sharded', 'sharded_1m') if k in d])"
done
