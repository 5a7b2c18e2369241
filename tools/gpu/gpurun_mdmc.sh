#!/bin/bash
# MCMD engine: GPU parity tests + stage timings (one box call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mdmc.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/mdmc_tests.log 2>&1 || { tail -40 gpurun_out/mdmc_tests.log; exit 1; }
tail -15 gpurun_out/mdmc_tests.log
timeout -k 10 200 python -u tools/mdmc_timing.py --ref > gpurun_out/mdmc_timing.log 2>&1 || { cat gpurun_out/mdmc_timing.log; exit 1; }
cat gpurun_out/mdmc_timing.log
if [ "${MDMC_PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mdmc_prof -o mdmc -- python3 -u tools/mdmc_timing.py \
      > gpurun_out/mdmc_prof.log 2>&1 || { tail -30 gpurun_out/mdmc_prof.log; exit 1; }
fi
