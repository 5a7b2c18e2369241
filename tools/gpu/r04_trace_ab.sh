#!/bin/bash
# Kernel trace of tools/force_ab.py (product library) at the given configs: per-kernel durations
# (block kernel, plan, sort, reduce) under rocprofv3 --kernel-trace --stats.
#   bash tools/gpu/r04_trace_ab.sh TAG [C3,C5,1M]
TAG=${1:-trace}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
MDQT_AB_CFGS=${2:-C3,C5,1M} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}" -o run -- python3 "$R/tools/force_ab.py" product > "$R/gpurun_out/${TAG}.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}.log"; exit 1; }
cd "$R"
python3 tools/prof_summary.py $(ls gpurun_out/${TAG}/*/*.db gpurun_out/${TAG}/*.db 2>/dev/null | head -1) > gpurun_out/${TAG}_kernel_stats.txt
exit 0
