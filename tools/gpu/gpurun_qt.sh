#!/bin/bash
# QT kernel iteration: parity suite of the MDQT path, then a C2 timing line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_qt.log 2>&1 || { tail -40 gpurun_out/pytest_qt.log; exit 1; }
tail -2 gpurun_out/pytest_qt.log
timeout -k 10 300 python bench.py --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines \
    --steps 200 --warmup 20 > gpurun_out/bench_qt.log 2>&1 || { tail -20 gpurun_out/bench_qt.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_qt.log').read().strip().splitlines()[-1]); k=d['config']['kernel_ms']; print(d['value'], round(d['ms_per_step']*1e3,2), 'us/step', 'sub', round(k['substeps_total']/k['substep_launches']*1e3,2), 'force', round(k['force_total']/k['force_launches']*1e3,2))"
