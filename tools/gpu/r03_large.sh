#!/bin/bash
# large configs: the block-kernel tests (sampled rows vs oracle, tail / far bounds on every ion) and
# the bench's large lines only (C3 MD-only, C5 sharded path, N = 1M with QT)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_large.log 2>&1
rc=$?
grep -E "^C[345]|^1M|^world|passed|failed|Error|^E " gpurun_out/pytest_large.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line > gpurun_out/bench_large.log 2>&1 || { tail -20 gpurun_out/bench_large.log; exit 1; }
tail -1 gpurun_out/bench_large.log > gpurun_out/bench_large.json
python3 -c "
import json; d=json.load(open('gpurun_out/bench_large.json'))
for k in ('md_only_c3','sharded','sharded_1m'):
    if k in d: print(k, round(d[k].get('ms_per_md_step'),2), round(d[k].get('force', {}).get('avg_ms'),2), d[k].get('force_tail'))
print('errors', d.get('secondary_errors'))"
