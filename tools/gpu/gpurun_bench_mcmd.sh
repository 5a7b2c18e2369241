#!/bin/bash
# MCMD tests + profile, then the full default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MDMC_PROF=1 bash tools/gpu/gpurun_mdmc.sh || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log > gpurun_out/bench_full.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_full.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('mcmd'), indent=1))"
