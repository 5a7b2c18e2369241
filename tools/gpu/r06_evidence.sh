#!/bin/bash
# round-6 evidence on the committed tree: GPU suite + smoke, the driver's bench command (timed),
# the same command under rocprofv3 --kernel-trace --stats, separate PMC passes on the C2 line, and
# the FETCH/WRITE calibration of the QT launch's access patterns (tools/fetch_calib.hip).
#   bash tools/gpu/r06_evidence.sh TAG     (outputs gpurun_out/<TAG>_*)
# (the large-N counters are a call of their own: tools/gpu/r06_large_pmc.sh)
TAG=${1:-r06}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "^C[345]|^1M|^world|^C2 headline|^MD step|passed|failed|Error|^E " gpurun_out/pytest_gpu.log | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
start=$(date +%s)
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
tail -1 gpurun_out/bench_full.log > gpurun_out/${TAG}_full_bench.json
grep "^BENCH_DETAIL " gpurun_out/bench_full.err | sed 's/^BENCH_DETAIL //' > gpurun_out/${TAG}_bench_detail.json
wc -c gpurun_out/${TAG}_full_bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --sharded-config none --million-config none --no-pump-lines --no-mcmd-lines --md-only-config none --no-e2e-line --no-replicas-line"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run -- python3 $B > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run -- python3 $B > "$R/gpurun_out/pmc_write.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc_sq" -o run -- python3 $B > "$R/gpurun_out/pmc_sq.log" 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/cal_fetch" -o run -- "$R/tools/fetch_calib" > "$R/gpurun_out/cal_fetch.log" 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/cal_write" -o run -- "$R/tools/fetch_calib" > "$R/gpurun_out/cal_write.log" 2>&1 || exit $?
cd "$R"
db() { ls gpurun_out/$1/*/*.db gpurun_out/$1/*.db 2>/dev/null | head -1; }
python3 tools/prof_summary.py $(db prof_$TAG) > gpurun_out/${TAG}_driver_cmd_kernel_stats.txt
python3 tools/prof_mainline.py $(db prof_$TAG) 24 > gpurun_out/${TAG}_driver_cmd_headline_kernels.txt 2>&1 || true
python3 tools/pmc_summary.py $(db cal_fetch) $(db cal_write) > gpurun_out/${TAG}_fetch_calib.json
cat gpurun_out/cal_fetch.log | grep "known bytes" > gpurun_out/${TAG}_fetch_calib_known.txt
FACT=$(python3 tools/calib_factors.py gpurun_out/${TAG}_fetch_calib.json gpurun_out/${TAG}_fetch_calib_known.txt)
echo "calibration factors (fetch write): $FACT"
python3 tools/pmc_summary.py $(db pmc_fetch) $(db pmc_write) $(db pmc_sq) --factors $FACT > gpurun_out/${TAG}_c2_pmc.json
grep "^{" gpurun_out/prof_$TAG.log | tail -1 > gpurun_out/${TAG}_driver_cmd_bench_under_rocprof.json || true
head -12 gpurun_out/${TAG}_driver_cmd_kernel_stats.txt
head -12 gpurun_out/${TAG}_driver_cmd_headline_kernels.txt
python3 tools/bench_brief.py gpurun_out/${TAG}_full_bench.json
