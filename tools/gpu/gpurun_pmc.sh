#!/bin/bash
# PMC passes (counters only, one group per pass, no tracing domains) on a short C2 bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o run -- python3 $B > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o run -- python3 $B > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_sq" -o run -- python3 $B > "$GRAFT_REPO_ROOT/gpurun_out/pmc_sq.log" 2>&1
echo "sq rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/pmc_sq.log"
