#!/bin/bash
# round 5: the weighted block ranges — GPU tests of the block scheme, the census model at C4/C5/1M,
# and per-rank block-kernel times of a world-8 in-process group at C5 (each rank alone on the GPU)
TAG=${1:-r05b}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -k "weighted or sharded or masked or block_work" -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "^C5|^world|passed|failed|Error|^E " gpurun_out/${TAG}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/load_balance.py c4 c5 c1m > gpurun_out/${TAG}_load_balance.json 2> gpurun_out/${TAG}_load_balance.err || { tail -5 gpurun_out/${TAG}_load_balance.err; exit 1; }
timeout -k 10 300 python3 -u tools/rank_balance.py c5 8 > gpurun_out/${TAG}_rank_balance_c5.json 2> gpurun_out/${TAG}_rank_balance.err || { tail -5 gpurun_out/${TAG}_rank_balance.err; exit 1; }
timeout -k 10 300 python3 -u tools/rank_balance.py c3 8 > gpurun_out/${TAG}_rank_balance_c3.json 2>> gpurun_out/${TAG}_rank_balance.err || { tail -5 gpurun_out/${TAG}_rank_balance.err; exit 1; }
cat gpurun_out/${TAG}_rank_balance.err
python3 -c "
import json
d=json.load(open('gpurun_out/${TAG}_load_balance.json'))
for k,v in d.items(): print(k, {x: round(y,4) for x,y in v['after_3_md_steps'].items() if 'world8' in x})"
