#!/bin/bash
# C2 headline + the jobs-per-GPU and end-to-end lines only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --sharded-config none --million-config none --no-mcmd-lines \
    --no-pump-lines --md-only-config none --steps 200 --warmup 20 > gpurun_out/bench_jobs.log 2>&1 || { tail -20 gpurun_out/bench_jobs.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_jobs.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('jobs_per_gpu'))); print(json.dumps(d.get('end_to_end'))); print(d.get('secondary_errors'))"
