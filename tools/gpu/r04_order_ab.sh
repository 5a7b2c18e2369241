#!/bin/bash
# A/B of the block kernel's workgroup order and count (tools/force_ab.py): run-major (product) vs
# block-major (expt/o0), and 4096 / 8192 / 16384 workgroups per rank (MDQT_N3B_WG).
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 tools/force_ab.py product || exit 1

  MDQT_N3B_WG=8192 timeout -k 10 200 python3 tools/force_ab.py wg8192 || exit 1
  MDQT_N3B_WG=16384 timeout -k 10 200 python3 tools/force_ab.py wg16384 || exit 1
done
exit 0
