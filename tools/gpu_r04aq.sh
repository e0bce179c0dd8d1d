#!/bin/bash
# uniform1k at 28 tiles per wave: stream tiles (dev product choice at
# threshold 24, ABLATE=0) against the CU schedule forced (ABLATE=15), both
# orders, 8 rounds each, to settle the threshold.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04aq}
mkdir -p "$O"
timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=15" --workload uniform1k --rounds 8 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab failed rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 23; }
timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=15" "SYNCR_CDC_ABLATE=0" --workload uniform1k --rounds 8 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab failed rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 23; }
cat "$O/${TAG}_dipab.jsonl"
echo done
