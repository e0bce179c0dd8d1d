#!/bin/bash
# Stream tiles vs the CU schedule on the shard sizes of config 4 at N = 2, 4, 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04aa}
mkdir -p "$O"
for w in shard8 shard4 shard2; do
  timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=15" "SYNCR_CDC_ABLATE=17" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 11; }
done
cat "$O/${TAG}_dipab.jsonl"
