#!/bin/bash
# full GPU suite, then the C2 bench with only the end-to-end (reference cadence) line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/gpurun_tests.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --sharded-config none --million-config none --no-mcmd-lines \
    --no-pump-lines --md-only-config none --steps 200 --warmup 20 > gpurun_out/bench_e2e.log 2>&1 || { tail -20 gpurun_out/bench_e2e.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_e2e.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print(json.dumps(d['end_to_end']))"
