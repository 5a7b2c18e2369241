#!/bin/bash
# the sharded lines through child processes: world 1 directly and under torchrun (nproc 1)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--steps 50 --warmup 5 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --no-e2e-line --no-replicas-line --sharded-in-child 1"
timeout -k 10 300 python bench.py $A > gpurun_out/child1.log 2>&1 || { tail -20 gpurun_out/child1.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 $A > gpurun_out/child2.log 2>&1 || { tail -20 gpurun_out/child2.log; exit 1; }
for f in child1 child2; do python3 -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], [(k, d[k]['ms_per_md_step']) for k in ('md_only_c3','sharded','sharded_1m') if k in d], d.get('secondary_errors'))"; done
