#!/bin/bash
# One GPU-box pass: parity tests, bench line, interleaved A/B of scan variants.
#   bash tools/gpu_check.sh [ab-variant ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$O/gpu_tests.log"; exit 11; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail -20 "$O/bench.err"; exit 12; }
cat "$O/bench.json"
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u tools/ab_bench.py "$@" --rounds 5 > "$O/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$O/ab.log"; exit 13; }
  cat "$O/ab.log"
fi
