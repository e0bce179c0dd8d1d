#!/bin/bash
# Full GPU test suite + smoke + the driver's bench command + the quick workload lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-full}
bash tools/gpu_round.sh $TAG || exit $?
bash tools/gpu_quick.sh ${TAG}q "kat" || exit $?
