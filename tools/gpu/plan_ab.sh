#!/bin/bash
# A/B of plan-kernel builds (tools/plan_ab.py), alternating, on one box:
#   bash tools/gpu/plan_ab.sh ROUNDS name1 name2 ...   (expt/<name>/lib/libmdqt.so; "base" = the product library)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$1; shift
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
    timeout -k 10 240 env $lib MDQT_AB_CFGS=${MDQT_AB_CFGS:-C3,C5,1M} python3 -u tools/plan_ab.py "$v" 3 \
      >> gpurun_out/plan_ab.txt 2>> gpurun_out/plan_ab.err || { echo "$v failed"; tail -5 gpurun_out/plan_ab.err; exit 1; }
  done
done
cat gpurun_out/plan_ab.txt
