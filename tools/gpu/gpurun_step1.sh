#!/bin/bash
# GPU pass: parity tests, smoke, bench (C2 + sharded C5 line), kernel-trace profiles of C2 and C5
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --sharded-config none --million-config none --qt-math 0 --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line > gpurun_out/bench_exact.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c5" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --sharded-config c5 --sharded-steps 2 --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line > "$GRAFT_REPO_ROOT/gpurun_out/prof_c5.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof1.log"
