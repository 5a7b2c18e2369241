#!/bin/bash
# round 2: large-config parity tests, full GPU suite, MD-step gap probe, QT/force stall counters (C2)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_large.log 2>&1
rc=$?
grep -E "^C[345]:|passed|failed|Error|assert" gpurun_out/pytest_large.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -u tools/gap_probe.py > gpurun_out/gap_probe.log 2>&1 || { tail -20 gpurun_out/gap_probe.log; exit 1; }
cat gpurun_out/gap_probe.log
rocprofv3 -L > gpurun_out/counters.txt 2>&1
B="$GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_a" -o run -- python3 $B > "$GRAFT_REPO_ROOT/gpurun_out/pmc_a.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_b" -o run -- python3 $B > "$GRAFT_REPO_ROOT/gpurun_out/pmc_b.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
python3 tools/pmc_summary.py $(ls gpurun_out/pmc_a/*/*.db gpurun_out/pmc_a/*.db 2>/dev/null | head -1) $(ls gpurun_out/pmc_b/*/*.db gpurun_out/pmc_b/*.db 2>/dev/null | head -1) > gpurun_out/pmc_r02a.json
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_r02a.json'))
for k,v in d.items():
    if 'lanes' in k or 'pairs_n3' in k: print(k[:50], {a: round(b) for a,b in v.items()})
"
