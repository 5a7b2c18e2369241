#!/bin/bash
# round 6: force-call A/B of the product against library variants copied to ab/<name>/libmdqt.so
# (git-ignored; expt/ does not travel to the GPU box), optionally after a pytest selection
#   TESTS="tests/a.py tests/b.py" KEXPR="x or y" VARIANTS="base nobar" CFGS=C3,C5,1M bash tools/gpu/r06_ab.sh TAG [rounds]
TAG=${1:-r06ab}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
export MDQT_AB_CFGS=${CFGS:-C3,C5,1M}
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 300 python3 tools/force_ab.py product || exit 1
  for v in ${VARIANTS:-}; do
    timeout -k 10 300 env MDQT_LIB=ab/$v/libmdqt.so python3 tools/force_ab.py $v || exit 1
  done
  for o in ${OPTS_VARIANTS:-}; do
    timeout -k 10 300 env MDQT_AB_OPTS=$o python3 tools/force_ab.py "product[$o]" || exit 1
  done
done 2>&1 | tee gpurun_out/${TAG}_force_ab.txt
