#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/ab.sh base wpe1 base wpe1 base wpe1 base wpe1
