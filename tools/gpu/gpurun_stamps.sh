#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
MDQT_LIB=$PWD/expt/stamps/lib/libmdqt.so timeout -k 10 120 python tools/n3_stamps.py 3500 && \
MDQT_LIB=$PWD/expt/stamps/lib/libmdqt.so timeout -k 10 120 python tools/n3_stamps.py 1000
