#!/bin/bash
# round 5: block-kernel correctness first (large configs, the block scheme, user inputs), then the
# force-call A/B of the product against the baseline tree (expt/basetree) and variants (expt/<name>)
#   VARIANTS="nodbuf noremat" bash tools/gpu/r05_ab.sh TAG [rounds]
TAG=${1:-r05ab}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -k "large or blocks or tail or sharded" -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_blocks.log 2>&1
rc=$?
grep -E "^C[345]|^1M|passed|failed|Error|^E " gpurun_out/${TAG}_blocks.log | head -30
[ $rc -eq 0 ] || exit $rc
BASE=${BASE:-basetree} VARIANTS="${VARIANTS:-}" bash tools/gpu/r04_force_ab.sh ${2:-2} 2>&1 | tee gpurun_out/${TAG}_force_ab.txt
