#!/bin/bash
# One-axis per-pair image (option force_ax1): optionally the GPU suite on the product build
# (TESTS=1), then the force-call A/B against the same library with force_ax1 0, alternating.
#   bash tools/gpu/r04_ax1_ab.sh [rounds]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/ax1_gpu.log 2>&1
  rc=$?
  grep -E "one-axis|passed|failed|Error|^E " gpurun_out/ax1_gpu.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${1:-2}); do
  timeout -k 10 200 python3 tools/force_ab.py product || exit 1
  timeout -k 10 200 env MDQT_AB_OPTS=force_ax1=0 python3 tools/force_ab.py force_ax1=0 || exit 1
done
exit 0
