#!/bin/bash
# round 2 first probe: f64 VALU microbenchmark, MD-step gap probe, kernel trace of the driver's bench command
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_f64 > gpurun_out/ubench.log 2>&1 || { tail -20 gpurun_out/ubench.log; exit 1; }
cat gpurun_out/ubench.log
timeout -k 10 180 python3 -u tools/gap_probe.py > gpurun_out/gap_probe.log 2>&1 || { tail -20 gpurun_out/gap_probe.log; exit 1; }
cat gpurun_out/gap_probe.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_drv" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pump-lines --no-mcmd-lines --md-only-config none --sharded-config none --million-config none --no-e2e-line --no-replicas-line > "$GRAFT_REPO_ROOT/gpurun_out/prof_drv.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_drv.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
tail -1 gpurun_out/prof_drv.log | cut -c1-400
python3 tools/kernel_gaps.py $(ls gpurun_out/prof_drv/*/*.db gpurun_out/prof_drv/*.db 2>/dev/null | head -1) --last 30 > gpurun_out/gaps.txt 2>&1
cat gpurun_out/gaps.txt | tail -45
