#!/bin/bash
# round 6: J-step balance estimates, Epotential-on-the-plan timing, the C2 tile-kernel variants (box-scaled
# form, split LDS reads) — their parity first, then the force-call A/B at C2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06c}
timeout -k 10 300 python3 tools/jstep_balance.py > gpurun_out/${T}_bal.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/pot_plan_check.py C3,C5,C4,1M 2 > gpurun_out/${T}_pot.txt 2>&1 || exit 1
for v in ${PARITY_VARIANTS:-ss}; do
  timeout -k 10 600 env MDQT_LIB=ab/$v/libmdqt.so python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "forces or newton3 or c2_headline or tile_split or md_steps or fused or overlapped" > gpurun_out/${T}_parity_$v.log 2>&1 || { tail -30 gpurun_out/${T}_parity_$v.log; exit 1; }
  tail -2 gpurun_out/${T}_parity_$v.log
done
CFGS=C2 VARIANTS="${AB_VARIANTS:-base scaled ss ldssplit}" bash tools/gpu/r06_ab.sh ${T} ${ROUNDS:-3}
