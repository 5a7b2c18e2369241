#!/bin/bash
# Stall counters of the block kernel, product library vs a baseline tree (expt/${BASE:-basetree}, a git worktree), at one
# config of tools/force_ab.py (diagnostic A/B; one rocprofv3 --pmc pass each).
#   bash tools/gpu/r04_diag_pmc.sh TAG [C3|C5|1M] [counters...]
TAG=${1:-diag}
CFG=${2:-C5}
shift 2
PMC=${@:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for v in product ${BASE:-basetree}; do
  cd /tmp
  if [ $v != product ]; then export MDQT_ROOT="$R/expt/$v"; else unset MDQT_ROOT; fi
  MDQT_AB_CFGS=$CFG timeout -s KILL 200 rocprofv3 --pmc $PMC -d "$R/gpurun_out/${TAG}_$v" -o run -- python3 "$R/tools/force_ab.py" $v > "$R/gpurun_out/${TAG}_$v.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_$v.log"; exit 1; }
  cd "$R"
  python3 tools/pmc_summary.py $(ls gpurun_out/${TAG}_$v/*/*.db gpurun_out/${TAG}_$v/*.db 2>/dev/null | head -1) > gpurun_out/${TAG}_$v.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$v.json'))
for k, x in d.items():
    if 'k_pairs_n3b' in k: print('$v', k, {c: round(val) for c, val in x.items()})"
done
exit 0
