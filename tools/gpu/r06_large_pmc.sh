#!/bin/bash
# Counter evidence for the large-N dominant kernel (k_pairs_n3b) at C3, C5 and N = 1M (VERDICT r03
# item 4): per config one bench.py run with only that line, under a kernel trace and three separate
# rocprofv3 --pmc passes (SQ + GRBM, FETCH_SIZE, WRITE_SIZE, VALU occupancy), summarised with the tree's source hash
# into gpurun_out/<TAG>_<cfg>_pmc.json (bench.py's large lines read the newest profiles/*_<cfg>_pmc.json).
#   bash tools/gpu/r06_large_pmc.sh TAG [cfgs...]
TAG=${1:-r06}
shift
CFGS=${@:-c3 c4 c5 c1m}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
BASE="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line --sharded-steps 1 --million-steps 1 --md-only-config none --sharded-config none --million-config none"
W=/tmp/large_pmc_$$                         # the databases stay on the box (gpurun_out/ is capped at 64 MiB)
mkdir -p $W
db() { ls $W/$1/*/*.db $W/$1/*.db 2>/dev/null | head -1; }
for cfg in $CFGS; do
  case $cfg in
    c3) B="$BASE --md-only-config c3" ;;
    c4) B="$BASE --md-only-config c4" ;;
    c5) B="$BASE --sharded-config c5" ;;
    c1m) B="$BASE --million-config c1m" ;;
    *) echo "unknown config $cfg"; exit 2 ;;
  esac
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$W/${TAG}_${cfg}_trace" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${cfg}_trace.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${cfg}_trace.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$W/${TAG}_${cfg}_sq" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${cfg}_sq.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${cfg}_sq.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$W/${TAG}_${cfg}_fetch" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${cfg}_fetch.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${cfg}_fetch.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$W/${TAG}_${cfg}_write" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${cfg}_write.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${cfg}_write.log"; exit 1; }
  # (round 6) a pass of VALU-occupancy counters: SQ_ACTIVE_INST_VALU (rocprofv3's VALUBusy = its sum / CUs /
  # GRBM_GUI_ACTIVE), dual issue, and the instruction mix (VALU_PMC= "" skips it)
  VALU_PMC=${VALU_PMC-"SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"}
  VDB=""
  if [ -n "${VALU_PMC:-}" ]; then
    timeout -s KILL 300 rocprofv3 --pmc $VALU_PMC -d "$W/${TAG}_${cfg}_valu" -o run -- python3 $B > "$R/gpurun_out/${TAG}_${cfg}_valu.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${cfg}_valu.log"; exit 1; }
    VDB=$(db ${TAG}_${cfg}_valu)
  fi
  cd "$R"
  python3 tools/pmc_summary.py $(db ${TAG}_${cfg}_sq) $(db ${TAG}_${cfg}_fetch) $(db ${TAG}_${cfg}_write) $VDB \
      --trace $(db ${TAG}_${cfg}_trace) --tag "bench.py ${cfg} line (steps 1): $B" > gpurun_out/${TAG}_${cfg}_pmc.json || exit 1
  python3 tools/prof_summary.py $(db ${TAG}_${cfg}_trace) > gpurun_out/${TAG}_${cfg}_kernel_stats.txt
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_${cfg}_pmc.json'))
k=max(tuple('void mdqt::k_pairs_n3b%s<1, false, false, %s>(mdqt::N3BArgs)' % (p, x) for p in ('', '_pw') for x in ('false', 'true')), key=lambda k: (d.get(k) or {}).get('dispatches', 0))
print('${cfg}', {x: d[k].get(x) for x in ('dispatches','duration_us','SQ_INSTS_VALU','SQ_WAVES','GRBM_GUI_ACTIVE','FETCH_SIZE','WRITE_SIZE')} if k in d else 'no n3b kernel')"
done
