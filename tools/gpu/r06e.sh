#!/bin/bash
# round 6: the paired-wave block kernel (k_pairs_n3b_pw) — block-scheme parity with it on (library built with
# MDQT_N3B_PAIRS_DEFAULT=1), then the force-call A/B against the product's 8-wave kernel
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06e}
for v in ${PARITY_VARIANTS:-pw5}; do
  timeout -k 10 900 env MDQT_LIB=ab/$v/libmdqt.so python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "large or blocks or tail or sharded or masked or block_work or epotential or scheme" > gpurun_out/${T}_parity_$v.log 2>&1 || { tail -40 gpurun_out/${T}_parity_$v.log; exit 1; }
  tail -2 gpurun_out/${T}_parity_$v.log
done
CFGS=${CFGS:-C3,C5,1M} VARIANTS="${AB_VARIANTS:-pw5 pw4}" bash tools/gpu/r06_ab.sh ${T} ${ROUNDS:-2}
