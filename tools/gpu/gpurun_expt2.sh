#!/bin/bash
# GPU: C2 bench per experimental variant (no parity suite: timing-only variants)
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-cur}; do
  MDQT_LIB=$PWD/expt/$v/lib/libmdqt.so timeout -k 10 300 python bench.py --no-cpu-baseline --sharded-config none --million-config none \
     --no-pump-lines --no-mcmd-lines --steps 200 --warmup 20 > gpurun_out/expt_$v.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/expt_$v.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print('$v', round(d['ms_per_step']*1e3,2), 'us/step', 'sub', round(k['substeps_total']/k['substep_launches']*1e3,2), 'force', round(k['force_total']/k['force_launches']*1e3,2))"
done
