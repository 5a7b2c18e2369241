cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MDQT_LIB=expt/stamps/lib/libmdqt.so timeout -k 10 120 python3 tools/n3_stamps.py > gpurun_out/n3_stamps.log 2>&1; cat gpurun_out/n3_stamps.log
