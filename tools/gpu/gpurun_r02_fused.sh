#!/bin/bash
# fused MD-step kernel: bit-identity tests, then C2 timing against the previous library
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or overlapped" > gpurun_out/pytest_fused.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_fused.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab.sh base prev base prev
