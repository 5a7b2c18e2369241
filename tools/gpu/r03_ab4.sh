#!/bin/bash
# round-3 A/B set 4 (C2): QT kernel scheduling / register budget variants
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/ab.sh base wpe1 schednone schedmmc base wpe1 schednone schedmmc
