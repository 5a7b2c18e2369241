#!/bin/bash
# round-3 A/B set 2: the block kernel's j-side step combining (MDQT_N3B_JCOMB 2 / 4) and the
# no-j-accumulation bound (timing only), on the large lines (C3, C5, N = 1M)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--steps 3 --warmup 1 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line --sharded-steps 3 --million-steps 2"
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  timeout -k 10 300 env $lib python3 bench.py $A > gpurun_out/abl_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abl_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1])
print('$v', 'C3 force ms', round(d['md_only_c3']['force']['avg_ms'],3), 'C5 force ms', round(d['sharded']['force']['avg_ms'],2), '1M ms/step', round(d['sharded_1m']['ms_per_md_step'],1))"
done
