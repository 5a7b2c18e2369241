#!/bin/bash
# round-3 start: GPU suite + smoke + the driver's bench command on the committed tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "^C[345]|^world|passed|failed|Error|^E " gpurun_out/pytest_gpu.log | head -40
echo "pytest rc=$rc"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log > gpurun_out/bench_full.json
python3 -c "
import json; d=json.load(open('gpurun_out/bench_full.json'))
print(d['value'], d['ms_per_step'], d['config']['kernel_ms'])
print('roof', {k: d['roofline'][k] for k in ('bound','achieved','frac','avg_launch_us','fp64_frac')})
for k in ('md_only_c3','sharded','sharded_1m'):
    if k in d: print(k, d[k].get('ms_per_md_step'), d[k].get('force', {}).get('avg_ms'))
print('errors', d.get('secondary_errors'))"
