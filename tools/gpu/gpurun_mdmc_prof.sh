#!/bin/bash
# MCMD engine: kernel trace of the stage timings
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mdmc_prof -o mdmc -- python3 -u tools/mdmc_timing.py \
    > gpurun_out/mdmc_prof.log 2>&1 || { tail -30 gpurun_out/mdmc_prof.log; exit 1; }
cat gpurun_out/mdmc_prof.log | grep -v "^W2\|rocprofv3" | tail -12
find gpurun_out/mdmc_prof -name "*kernel_stats.csv" | head -3
