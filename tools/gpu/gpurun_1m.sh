#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pump-lines --no-mcmd-lines \
    --sharded-config none --million-config c1m > gpurun_out/bench_1m.log 2>&1 || { tail -30 gpurun_out/bench_1m.log; exit 1; }
tail -1 gpurun_out/bench_1m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['sharded_1m']))"
