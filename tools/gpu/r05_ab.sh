#!/bin/bash
# round 5: block-kernel correctness first (large configs, the block scheme, user inputs), then the
# force-call A/B of the product against the baseline tree (expt/basetree), variants (expt/<name>) and
# the product with engine options (OPTS_VARIANTS="force_reduce_mask=0 ...")
#   VARIANTS="nodbuf noremat" bash tools/gpu/r05_ab.sh TAG [rounds]
TAG=${1:-r05ab}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -k "large or blocks or tail or sharded or masked or block_work" -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_blocks.log 2>&1
rc=$?
grep -E "^C[345]|^1M|passed|failed|Error|^E " gpurun_out/${TAG}_blocks.log | head -30
[ $rc -eq 0 ] || exit $rc
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 200 python3 tools/force_ab.py product || exit 1
  timeout -k 10 200 env MDQT_ROOT="$R/expt/${BASE:-basetree}" python3 tools/force_ab.py ${BASE:-basetree} || exit 1
  for v in ${VARIANTS:-}; do
    timeout -k 10 200 env MDQT_LIB=expt/$v/lib/libmdqt.so python3 tools/force_ab.py $v || exit 1
  done
  for o in ${OPTS_VARIANTS:-}; do
    timeout -k 10 200 env MDQT_AB_OPTS=$o python3 tools/force_ab.py "product[$o]" || exit 1
  done
done 2>&1 | tee gpurun_out/${TAG}_force_ab.txt
