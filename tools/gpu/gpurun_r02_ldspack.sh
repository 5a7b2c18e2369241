#!/bin/bash
# the tile kernel's packed LDS (J tile at offset 0): force parity tests, then A/B vs the old layout
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "newton3 or force or epot or momentum or fused or overlap" > gpurun_out/ldspack_tests.log 2>&1 || { tail -20 gpurun_out/ldspack_tests.log; exit 1; }
tail -1 gpurun_out/ldspack_tests.log
bash tools/gpu/ab.sh base nopack base nopack
