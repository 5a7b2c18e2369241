#!/bin/bash
# round 5: block-kernel issue priority (expt/prio) and the thread-per-ion QT kernel's occupancy
# (expt/qtr2, expt/qtr3) against the product, alternating
#   bash tools/gpu/r05_ab2.sh TAG [rounds]
TAG=${1:-r05ab2}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 200 python3 tools/force_ab.py product || exit 1
  for v in ${FVARIANTS:-prio}; do
    timeout -k 10 200 env MDQT_LIB=expt/$v/lib/libmdqt.so python3 tools/force_ab.py $v || exit 1
  done
  timeout -k 10 200 python3 tools/qt_ab.py product || exit 1
  for v in ${QVARIANTS:-qtr2 qtr3}; do
    timeout -k 10 200 env MDQT_LIB=expt/$v/lib/libmdqt.so python3 tools/qt_ab.py $v || exit 1
  done
done 2>&1 | tee gpurun_out/${TAG}.txt
