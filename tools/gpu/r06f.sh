#!/bin/bash
# round 6: the whole GPU suite and smoke on the current tree, then the driver's bench command with its
# detail line kept, and the rocprofv3 kernel trace of the same command
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06f}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/${T}_pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { cat gpurun_out/${T}_smoke.txt; exit 1; }
cat gpurun_out/${T}_smoke.txt
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
tail -c 3000 gpurun_out/${T}_bench.out
