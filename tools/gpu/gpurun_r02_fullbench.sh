#!/bin/bash
# the driver's default bench command (full line incl. secondary items), timed
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
echo "wall $(( $(date +%s) - start )) s"
tail -1 gpurun_out/bench_full.log > gpurun_out/bench_full.json
python3 -c "
import json; d=json.load(open('gpurun_out/bench_full.json'))
print(d['value'], d['ms_per_step'], d['config']['kernel_ms'])
print('roof', {k: d['roofline'][k] for k in ('bound','achieved','frac','avg_launch_us','fp64_frac')})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['single_thread']['value'])
for k in ('md_only_c3','sharded','sharded_1m'):
    if k in d: print(k, d[k]['ms_per_md_step'], d[k].get('cpu_baseline',{}).get('value'))
print('errors', d.get('secondary_errors'))"
