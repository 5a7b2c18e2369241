#!/bin/bash
# round-3 A/B set 3 (C2): the jump draws precomputed in the QT prologue, and the no-jump bound
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/ab.sh base jpre nojump base jpre nojump
