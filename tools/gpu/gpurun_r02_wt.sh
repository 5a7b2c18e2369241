#!/bin/bash
# write-through slot / QT state stores: GPU suite + smoke, then A/B vs plain stores (C2 line)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wt_tests.log 2>&1 || { tail -20 gpurun_out/wt_tests.log; exit 1; }
tail -1 gpurun_out/wt_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
bash tools/gpu/ab.sh base plain base plain
