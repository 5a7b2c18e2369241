#!/bin/bash
# A/B kernel timing of library variants built by tools/expt_build.sh (C2 line only):
#   bash tools/gpu/ab.sh base nojacc w8 ...   (base = the product library)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--steps 200 --warmup 20 --timing-period 8 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  timeout -k 10 200 env $lib python3 bench.py $A > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print('$v', round(d['value']/1e9,4), 'step', round(d['ms_per_step']*1e3,2), 'force', round(k['force_total']/k['force_launches']*1e3,2), 'qt', round(k['substeps_total']/k['substep_launches']*1e3,2))"
done
