#!/bin/bash
# Where the stream-tile scan loses on the dense workload: all-periodic corpus A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04w}
mkdir -p "$O"
timeout -k 10 300 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=8" --workload periodic --rounds 2 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 11; }
cat "$O/${TAG}_dipab.jsonl"
