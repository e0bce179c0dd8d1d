#!/bin/bash
# uniform1k (28 tiles per wave): the CU schedule (product) vs stream tiles forced.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04ao}
mkdir -p "$O"
timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=17" --workload uniform1k --rounds 6 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 11; }
cat "$O/${TAG}_dipab.jsonl"
