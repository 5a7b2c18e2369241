#!/bin/bash
# full GPU parity suite + smoke + MCMD stage timings + C2 timing line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/gpurun_tests.sh || exit $?
timeout -k 10 200 python -u tools/mdmc_timing.py > gpurun_out/mdmc_timing.log 2>&1 || { cat gpurun_out/mdmc_timing.log; exit 1; }
cat gpurun_out/mdmc_timing.log
timeout -k 10 300 python bench.py --no-cpu-baseline --sharded-config none --million-config none --no-mcmd-lines --md-only-config none --no-e2e-line \
    --steps 200 --warmup 20 > gpurun_out/bench_qt.log 2>&1 || { tail -20 gpurun_out/bench_qt.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_qt.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print(d['value'], round(d['ms_per_step']*1e3,2), 'us/step', 'sub', round(k['substeps_total']/k['substep_launches']*1e3,2), 'force', round(k['force_total']/k['force_launches']*1e3,2)); print([ (p['qt_model'], round(p['ms_per_md_step']*1e3,2)) for p in d['pump_models']])"
