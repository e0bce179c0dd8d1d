#!/bin/bash
# Stream tiles with the tile-granular tail (dev SYNCR_CDC_ABLATE=18): the GPU suite
# with it forced, timelines, and A/B against the product stream tiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04am}
mkdir -p "$O"
SYNCR_TEST_DEV_LIBRARY=1 SYNCR_CDC_ABLATE=18 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not product_ignores and not capi" > "$O/${TAG}_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 10; }
tail -1 "$O/${TAG}_tests.log"
for w in zipf10k shard8; do
  SYNCR_CDC_ABLATE=18 timeout -k 10 120 python -u tools/scan_timeline.py --workload $w > "$O/${TAG}_tl_${w}.json" 2>>"$O/${TAG}_tl.err" || { echo "timeline $w rc=$?"; tail -20 "$O/${TAG}_tl.err"; exit 21; }
  python3 -c "
import json; d=json.load(open('$O/${TAG}_tl_${w}.json'))
x=d['last_of_25']; print('$w', x['ends_us'], x['first_land_us'], x['resolve_start_after_scan_us'])"
done
for w in zipf10k shard8 shard4; do
  timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=18" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 11; }
done
cat "$O/${TAG}_dipab.jsonl"
