#!/bin/bash
# round 5: GPU suite (new user-input parity file first) + smoke + the driver's bench command
#   bash tools/gpu/r05_suite.sh TAG     (outputs gpurun_out/<TAG>_*)
TAG=${1:-r05}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_user_inputs.py -x -v -rP --timeout 120 --timeout-method thread > gpurun_out/${TAG}_user_inputs.log 2>&1
rc=$?
grep -E "rng_mode|passed|failed|Error|^E " gpurun_out/${TAG}_user_inputs.log | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
grep -E "^C[345]|^1M|^world|^C2 headline|passed|failed|Error|^E " gpurun_out/${TAG}_pytest_gpu.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
start=$(date +%s)
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.out 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
tail -1 gpurun_out/${TAG}_bench.out > gpurun_out/${TAG}_full_bench.json
grep "^BENCH_DETAIL " gpurun_out/${TAG}_bench.err | sed 's/^BENCH_DETAIL //' > gpurun_out/${TAG}_bench_detail.json
wc -c gpurun_out/${TAG}_full_bench.json
python3 tools/bench_brief.py gpurun_out/${TAG}_full_bench.json
timeout -k 10 300 python3 -u tools/load_balance.py c4 c5 c1m > gpurun_out/${TAG}_load_balance.json 2> gpurun_out/${TAG}_load_balance.err || { tail -20 gpurun_out/${TAG}_load_balance.err; exit 1; }
cat gpurun_out/${TAG}_load_balance.err
