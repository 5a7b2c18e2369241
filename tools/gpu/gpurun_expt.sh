#!/bin/bash
# GPU: parity suite on the product build, then C2 bench per experimental variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-cur}; do
  MDQT_LIB=$PWD/expt/$v/lib/libmdqt.so timeout -k 10 300 python bench.py --no-cpu-baseline --sharded-config none --million-config none \
     --steps 200 --warmup 20 > gpurun_out/expt_$v.log 2>&1 || exit $?
  echo "$v done"
done
