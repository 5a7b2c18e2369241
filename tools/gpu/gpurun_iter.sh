#!/bin/bash
# GPU iteration pass: parity suite, short C2 bench lines, kernel-trace summary of the C2 bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --sharded-config none --million-config none ${BENCH_ARGS} > gpurun_out/bench_iter.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_iter" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --sharded-config none --million-config none ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof_iter.log" 2>&1 || exit $?
exit $rc
