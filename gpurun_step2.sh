#!/bin/bash
# tests + bench + kernel trace, then PMC passes (counters only)
cd "$GRAFT_REPO_ROOT" || exit 1
bash gpurun_step1.sh || exit $?
bash gpurun_pmc.sh
