#!/bin/bash
# per-wave stamps of the production QT launch (diagnostic build expt/qtstamps)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MDQT_LIB=expt/qtstamps/lib/libmdqt.so timeout -k 10 120 python3 tools/qt_stamps.py > gpurun_out/diag_qt_stamps.txt 2>&1 || { cat gpurun_out/diag_qt_stamps.txt; exit 1; }
cat gpurun_out/diag_qt_stamps.txt
