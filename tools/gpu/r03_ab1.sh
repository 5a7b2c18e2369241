#!/bin/bash
# round-3 A/B set 1: QT layout (2 / 1 ions per wave), phase rotation (timing only), nt slot loads,
# the old wrap; each variant twice, alternating (tools/gpu/ab.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/ab.sh base rows2 phaserot ntslot wrapold base rows2 phaserot ntslot wrapold rows1
