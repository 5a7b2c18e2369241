#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log > gpurun_out/bench_full.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_full.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d['mcmd']['qt_tagging'])); print(d['mcmd']['main_estimate_s'])"
