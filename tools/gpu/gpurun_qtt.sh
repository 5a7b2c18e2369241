#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mdmc_qt.py tests/test_mdmc.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/qtt_tests.log 2>&1 || { tail -50 gpurun_out/qtt_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/qtt_tests.log | tail -25
