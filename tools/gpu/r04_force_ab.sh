#!/bin/bash
# A/B of the block-kernel variants at C3, C5, N = 1M (tools/force_ab.py): the product library, the
# baseline tree (expt/basetree: a git worktree with its own build) and diagnostic builds (expt/<name>), alternating.
#   bash tools/gpu/r04_force_ab.sh [rounds]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for i in $(seq 1 ${1:-2}); do
  timeout -k 10 200 python3 tools/force_ab.py product || exit 1
  timeout -k 10 200 env MDQT_ROOT="$R/expt/${BASE:-basetree}" python3 tools/force_ab.py ${BASE:-basetree} || exit 1
  for v in ${VARIANTS:-}; do
    [ -f expt/$v/lib/libmdqt.so ] && { timeout -k 10 200 env MDQT_LIB=expt/$v/lib/libmdqt.so python3 tools/force_ab.py $v || exit 1; }
  done
done
exit 0
