#!/bin/bash
# Profiles of this round's code on one box: the driver's command under the
# kernel trace + PMC passes (headline corpus), the same for the adversarial
# dense workload, then the one-GPU strong-scaling rehearsal.
#   bash tools/gpu_prof_round.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03}
bash tools/prof.sh ${TAG} || exit 21
bash tools/prof.sh ${TAG}dense --workload dense || exit 22
bash tools/gpu_rehearsal.sh ${TAG}_rehearsal || exit 23
echo all-done
