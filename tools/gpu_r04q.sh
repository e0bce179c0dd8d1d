#!/bin/bash
# Cost of the scan-timing events inside the timed step loop (tools/event_overhead.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04q}
mkdir -p "$O"
for w in uniform1k shard8 zipf10k; do
  timeout -k 10 180 python -u tools/event_overhead.py --workload $w --rounds 3 >> "$O/${TAG}_events.jsonl" 2>> "$O/${TAG}_events.err" || { echo "$w rc=$?"; tail -20 "$O/${TAG}_events.err"; exit 11; }
done
cat "$O/${TAG}_events.jsonl"
