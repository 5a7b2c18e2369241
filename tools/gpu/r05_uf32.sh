#!/bin/bash
# round 5: the f32 ultra-far form relative to J's first ion — large-config GPU tests, then the force-call
# A/B against the previous product library (expt/r05f) and variants (expt/<name>) at C4 and N = 1M (the
# configurations with an f32 shell), alternating
#   VARIANTS="uf32pk" bash tools/gpu/r05_uf32.sh TAG [rounds]
TAG=${1:-r05uf32}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -q -rP --timeout 600 --timeout-method thread > gpurun_out/${TAG}_large.log 2>&1
rc=$?
grep -E "^C[345]|^1M|N=|passed|failed|Error|^E " gpurun_out/${TAG}_large.log | head -40
[ $rc -eq 0 ] || exit $rc
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 300 env MDQT_AB_CFGS=C4,1M python3 tools/force_ab.py product || exit 1
  timeout -k 10 300 env MDQT_AB_CFGS=C4,1M MDQT_LIB=expt/${BASE:-r05f}/lib/libmdqt.so python3 tools/force_ab.py ${BASE:-r05f} || exit 1
  for v in ${VARIANTS:-}; do
    timeout -k 10 300 env MDQT_AB_CFGS=C4,1M MDQT_LIB=expt/$v/lib/libmdqt.so python3 tools/force_ab.py $v || exit 1
  done
done 2>&1 | tee gpurun_out/${TAG}_force_ab.txt
