#!/bin/bash
# spatial order: large-config tests, block-pair tests, sharded/MD-only force timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -k "large or spatial or newton3" -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_large.log 2>&1
rc=$?
grep -E "^C[345]|passed|failed|Error|assert" gpurun_out/pytest_large.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line > gpurun_out/bench_big.log 2>&1 || { tail -5 gpurun_out/bench_big.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_big.log').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step']*1e3)
for k in ('md_only_c3','sharded','sharded_1m'):
    if k in d: print(k, d[k]['ms_per_md_step'], d[k]['force'])
print(d.get('secondary_errors'))"
