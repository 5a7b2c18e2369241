#!/bin/bash
# round-end confirmation: GPU parity suite + smoke, the default bench line, kernel-trace summary of a C2 bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/gpurun_tests.sh || exit $?
bash tools/gpu/gpurun_bench.sh || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_final" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline --sharded-config c5 --million-config none --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line > "$GRAFT_REPO_ROOT/gpurun_out/prof_final.log" 2>&1 || exit $?
tail -1 "$GRAFT_REPO_ROOT/gpurun_out/prof_final.log" | cut -c1-300
