#!/bin/bash
# Stream-tile scan (product for large batches) vs the round-3 tile scan with
# dynamic groups (dev SYNCR_CDC_ABLATE=8) on the headline and the dense workload,
# after the ST kernel's parity on the GPU suite (product library).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04u}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 10; }
tail -1 "$O/${TAG}_tests.log"
for w in zipf10k dense; do
  timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=8" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 11; }
done
cat "$O/${TAG}_dipab.jsonl"
