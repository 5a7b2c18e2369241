#!/bin/bash
# force-path GPU tests: large configs, spatial order, sharded blocks, force parity
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -m gpu -x -q -rP --timeout 400 --timeout-method thread -k "large or spatial or sharded or force or newton or n3" > gpurun_out/pytest_force.log 2>&1
rc=$?
grep -E "^C[345]|world|sorted|passed|failed|Error|assert" gpurun_out/pytest_force.log | head -40
exit $rc
