#!/bin/bash
# GPU tests, then dev-library A/Bs given as "workload|variant variant ..." args.
#   bash tools/gpu_check_ab.sh TAG "dense|SYNCR_CDC_RESOLVE_PF=2 SYNCR_CDC_RESOLVE_PF=8" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
TAG=$1
shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/${TAG}_tests.log; exit 11; }
tail -2 $O/${TAG}_tests.log
n=0
for spec in "$@"; do
  n=$((n+1))
  w=${spec%%|*}
  v=${spec#*|}
  timeout -k 10 300 python -u tools/ab_bench.py $v --workload $w --rounds 5 > $O/${TAG}_ab$n.log 2>&1 || { tail -20 $O/${TAG}_ab$n.log; exit 12; }
  echo "== $w"; grep -E "scan med|DIFFER" $O/${TAG}_ab$n.log
done
