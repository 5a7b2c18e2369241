#!/bin/bash
# A/B of the block kernel's workgroups per rank (engine option MDQT_N3B_WG, default 16384)
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  for wg in 16384 8192 32768 65536; do
    MDQT_N3B_WG=$wg timeout -k 10 200 python3 tools/force_ab.py wg$wg || exit 1
  done
done
exit 0
