#!/bin/bash
# Instruction-fetch counters of the block kernel (k_pairs_n3b: ~92 KB of code, more than the
# instruction cache) at C3 / C5: does the six-level dispatch stall on instruction fetch?
#   bash tools/gpu/r04_icache_pmc.sh TAG [cfgs...]      (outputs gpurun_out/<TAG>_<cfg>_icache.json)
TAG=${1:-r04}
shift
CFGS=${@:-c3 c5}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
BASE="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line --sharded-steps 1 --million-steps 1 --md-only-config none --sharded-config none --million-config none"
W=/tmp/icache_pmc_$$
mkdir -p $W
db() { ls $W/$1/*/*.db $W/$1/*.db 2>/dev/null | head -1; }
cd /tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters_avail.txt" 2>&1 || true
grep -o "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" "$R/gpurun_out/${TAG}_counters_avail.txt" | sort -u | tr '\n' ' '
echo
for cfg in $CFGS; do
  case $cfg in
    c3) B="$BASE --md-only-config c3" ;;
    c5) B="$BASE --sharded-config c5" ;;
    c1m) B="$BASE --million-config c1m" ;;
    *) echo "unknown config $cfg"; exit 2 ;;
  esac
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$W/${TAG}_${cfg}_ic" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${cfg}_ic.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${cfg}_ic.log"; exit 1; }
  cd "$R"
  python3 tools/pmc_summary.py $(db ${TAG}_${cfg}_ic) --tag "bench.py ${cfg} line (steps 1): icache" > gpurun_out/${TAG}_${cfg}_icache.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_${cfg}_icache.json'))
k=max(('void mdqt::k_pairs_n3b<1, false, false, false>(mdqt::N3BArgs)', 'void mdqt::k_pairs_n3b<1, false, false, true>(mdqt::N3BArgs)'), key=lambda k: (d.get(k) or {}).get('dispatches', 0))
print('${cfg}', d.get(k, 'no n3b kernel'))"
done
