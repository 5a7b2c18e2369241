#!/bin/bash
# round 2 evidence: the driver's exact bench command under rocprofv3 --kernel-trace --stats, the
# same command's JSON line, and separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) on the C2 line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r02" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$R/gpurun_out/prof_r02.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_r02.log"; exit 1; }
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run -- python3 $B > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run -- python3 $B > "$R/gpurun_out/pmc_write.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc_sq" -o run -- python3 $B > "$R/gpurun_out/pmc_sq.log" 2>&1 || exit $?
cd "$R"
python3 tools/prof_summary.py $(ls gpurun_out/prof_r02/*/*.db gpurun_out/prof_r02/*.db 2>/dev/null | head -1) > gpurun_out/r02_driver_cmd_kernel_stats.txt
python3 tools/pmc_summary.py $(ls gpurun_out/pmc_fetch/*/*.db gpurun_out/pmc_fetch/*.db 2>/dev/null | head -1) $(ls gpurun_out/pmc_write/*/*.db gpurun_out/pmc_write/*.db 2>/dev/null | head -1) $(ls gpurun_out/pmc_sq/*/*.db gpurun_out/pmc_sq/*.db 2>/dev/null | head -1) > gpurun_out/r02_c2_pmc.json
grep "^{" gpurun_out/prof_r02.log | tail -1 > gpurun_out/r02_driver_cmd_bench.json
head -12 gpurun_out/r02_driver_cmd_kernel_stats.txt
python3 -c "
import json; d=json.load(open('gpurun_out/r02_c2_pmc.json'))
for k,v in d.items():
    if 'lanes' in k or 'pairs_n3' in k: print(k[:60], {a: round(b) for a,b in v.items()})
b=json.load(open('gpurun_out/r02_driver_cmd_bench.json')); print(b['value'], b['roofline'])"
