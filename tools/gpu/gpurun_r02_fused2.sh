#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 env MDQT_LIB=expt/mdstamps/lib/libmdqt.so python3 tools/md_stamps.py || exit 1
timeout -k 10 120 python3 tools/sig_probe.py || exit 1
