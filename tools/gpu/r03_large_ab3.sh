#!/bin/bash
# large-N tests on the product library, then the large bench lines alternating with variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_large.log 2>&1
rc=$?
grep -E "^C[345] N=|passed|failed|Error|^E " gpurun_out/pytest_large.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/r03_large_ab2.sh "$@"
