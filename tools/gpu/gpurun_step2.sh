#!/bin/bash
# tests + bench + kernel trace, then PMC passes (counters only)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/gpurun_step1.sh || exit $?
bash tools/gpu/gpurun_pmc.sh
