#!/bin/bash
# QT prologue iteration: stamps, GPU parity suite, short C2 bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
MDQT_LIB=$PWD/expt/qtstamps/lib/libmdqt.so timeout -k 10 120 python tools/qt_stamps.py 3500 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line > gpurun_out/bench_c2.log 2>&1 || { tail -5 gpurun_out/bench_c2.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c2.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']*1e3, d['config']['kernel_ms'], d['roofline']['avg_launch_us'])"
