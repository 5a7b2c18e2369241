#!/bin/bash
# kernel trace of the end-to-end line (mdqt_run at the reference cadence) only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$R/gpurun_out/prof_e2e" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-replicas-line > "$R/gpurun_out/prof_e2e.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_e2e.log"; exit 1; }
cd "$R"
python3 tools/prof_summary.py $(ls gpurun_out/prof_e2e/*/*.db gpurun_out/prof_e2e/*.db 2>/dev/null | head -1) | head -25
