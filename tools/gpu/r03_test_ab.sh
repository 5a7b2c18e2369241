#!/bin/bash
# GPU suite on the product library, then an A/B of the product against expt variants (C2 line)
#   bash tools/gpu/r03_test_ab.sh variant ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "^C2 headline|passed|failed|Error|^E " gpurun_out/pytest_gpu.log | head -30
[ $rc -eq 0 ] || exit $rc
args=""
for v in "$@"; do args="$args base $v"; done
bash tools/gpu/ab.sh $args base
