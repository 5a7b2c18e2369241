#!/bin/bash
# A/B of library variants on the large-N force lines (C3 MD-only, C5 sharded on one GPU):
#   bash tools/gpu/ab_large.sh base prev ...   (base = the product library, others expt/<name>)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--steps 5 --warmup 2 --no-cpu-baseline --million-config none --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line"
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  timeout -k 10 300 env $lib python3 bench.py $A > gpurun_out/abl_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abl_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1])
print('$v', 'C3 force ms', round(d['md_only_c3']['force']['avg_ms'],3), 'frac', round(d['md_only_c3']['force']['fp64_frac'],3), 'C5 force ms', round(d['sharded']['force']['avg_ms'],2))"
done
