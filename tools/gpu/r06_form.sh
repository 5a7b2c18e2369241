#!/bin/bash
# round 6, force_form_mode: a pytest selection (failures reported, not fatal), then the force-call A/B
# of the product against force_form_mode 0
#   TESTS="tests/test_gpu_large.py" KEXPR="..." CFGS=C3,C5,C4,1M bash tools/gpu/r06_form.sh TAG [rounds]
TAG=${1:-r06form}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -v -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | tail -40
  tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -le 1 ] || exit $rc                  # a crash or time limit: nothing more on the GPU
fi
export MDQT_AB_CFGS=${CFGS:-C3,C5,C4,1M}
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 300 python3 tools/force_ab.py product || exit 1
  for o in ${OPTS_VARIANTS:-force_form_mode=0}; do
    timeout -k 10 300 env MDQT_AB_OPTS=$o python3 tools/force_ab.py "product[$o]" || exit 1
  done
done 2>&1 | tee gpurun_out/${TAG}_force_ab.txt
