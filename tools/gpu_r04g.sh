#!/bin/bash
# The fine per-region scan schedule (dev SYNCR_CDC_ABLATE=17): parity of the
# whole GPU suite on the dev library with it forced, then A/B against the
# product schedules in the driver's condition, and its timeline.
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
for w in uniform1k zipf10k; do
  SYNCR_CDC_ABLATE=17 timeout -k 10 120 python -u tools/scan_timeline.py --workload $w > "$O/${TAG}_tl_${w}_a17.json" 2>>"$O/${TAG}_tl.err" || { echo "timeline $w failed rc=$?"; tail -20 "$O/${TAG}_tl.err"; exit 21; }
done
echo done
