#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_r04b.sh r04b || exit $?
bash tools/gpu_r04c.sh r04c || exit $?
