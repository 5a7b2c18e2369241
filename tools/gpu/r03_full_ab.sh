#!/bin/bash
# GPU suite, then C2 A/B (ab.sh) and large-line A/B (r03_large_ab2.sh) of the product against variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "^C2 headline|^C[345] N=|passed|failed|Error|^E " gpurun_out/pytest_gpu.log | head -30
[ $rc -eq 0 ] || exit $rc
args=""
for v in "$@"; do args="$args base $v"; done
bash tools/gpu/ab.sh $args base || exit 1
bash tools/gpu/r03_large_ab2.sh $args
