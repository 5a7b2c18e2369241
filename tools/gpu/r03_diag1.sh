#!/bin/bash
# round-3 diagnostics at C2: per-workgroup stamps of the force tile kernel, per-wave stamps of the
# QT lane kernel (diagnostic builds expt/stamps, expt/qtstamps), and the SQ wait breakdown of both
# kernels (one PMC pass, the C2 bench line only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
MDQT_LIB=expt/stamps/lib/libmdqt.so timeout -k 10 120 python3 tools/n3_stamps.py > gpurun_out/diag_n3_stamps.txt 2>&1 || { cat gpurun_out/diag_n3_stamps.txt; exit 1; }
cat gpurun_out/diag_n3_stamps.txt
MDQT_LIB=expt/qtstamps/lib/libmdqt.so timeout -k 10 120 python3 tools/qt_stamps.py > gpurun_out/diag_qt_stamps.txt 2>&1 || { cat gpurun_out/diag_qt_stamps.txt; exit 1; }
cat gpurun_out/diag_qt_stamps.txt
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -d "$R/gpurun_out/pmc_wait" -o run -- python3 $B > "$R/gpurun_out/pmc_wait.log" 2>&1 || exit $?
cd "$R"
db=$(ls gpurun_out/pmc_wait/*/*.db gpurun_out/pmc_wait/*.db 2>/dev/null | head -1)
python3 tools/pmc_summary.py $db > gpurun_out/diag_pmc_wait.json
python3 -c "
import json; d=json.load(open('gpurun_out/diag_pmc_wait.json'))
for k, v in d.items():
    if 'pairs_n3<1' in k or 'lanes_im' in k:
        w = v['SQ_WAVES']
        print(k[:60], {c: round(x / w, 1) for c, x in v.items() if c.startswith('SQ_')})"
