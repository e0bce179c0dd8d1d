#!/bin/bash
# The stream-tile scan (dev SYNCR_CDC_ABLATE=17): parity of the whole GPU
# suite on the dev library with it forced, then A/B against the product scan
# and the no-warm-up/no-halo timing ablation in the driver's condition.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04c}
mkdir -p "$O"
SYNCR_TEST_DEV_LIBRARY=1 SYNCR_CDC_ABLATE=17 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not product_ignores and not capi" > "$O/${TAG}_tests_fine.log" 2>&1 || { echo "fine tests failed rc=$?"; tail -30 "$O/${TAG}_tests_fine.log"; exit 11; }
tail -2 "$O/${TAG}_tests_fine.log"
for w in uniform1k shard8 zipf10k; do
  timeout -k 10 180 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=17" "SYNCR_CDC_ABLATE=13" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w failed rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 23; }
done
cat "$O/${TAG}_dipab.jsonl"
echo done
