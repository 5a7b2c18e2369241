#!/bin/bash
# dispatch rate of a C2-tile-kernel-shaped grid (tools/dispatch_probe.hip) and the force kernel's
# per-workgroup stamps against the tile-pair order (expt/stamps)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 tools/dispatch_probe 1596 0 100 1000 4000 > gpurun_out/diag_dispatch.txt 2>&1 || { cat gpurun_out/diag_dispatch.txt; exit 1; }
timeout -k 10 60 tools/dispatch_probe 256 0 4000 >> gpurun_out/diag_dispatch.txt 2>&1 || { cat gpurun_out/diag_dispatch.txt; exit 1; }
timeout -k 10 60 tools/dispatch_probe 4096 0 4000 >> gpurun_out/diag_dispatch.txt 2>&1 || { cat gpurun_out/diag_dispatch.txt; exit 1; }
cat gpurun_out/diag_dispatch.txt
MDQT_LIB=expt/stamps/lib/libmdqt.so timeout -k 10 120 python3 tools/n3_stamps.py > gpurun_out/diag_n3_stamps.txt 2>&1 || { cat gpurun_out/diag_n3_stamps.txt; exit 1; }
cat gpurun_out/diag_n3_stamps.txt
