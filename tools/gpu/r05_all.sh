#!/bin/bash
# round 5: A/B (r05_ab.sh) then the whole suite + bench + load balance (r05_suite.sh)
TAG=${1:-r05}
cd "$GRAFT_REPO_ROOT" || exit 1
VARIANTS="${VARIANTS:-}" bash tools/gpu/r05_ab.sh ${TAG}ab ${ROUNDS:-2} || exit $?
bash tools/gpu/r05_suite.sh $TAG
