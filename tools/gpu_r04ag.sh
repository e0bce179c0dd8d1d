#!/bin/bash
# Stream-tile scan timelines (dev stamps): how far apart the waves end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04ag}
mkdir -p "$O"
for w in zipf10k shard8; do
  timeout -k 10 120 python -u tools/scan_timeline.py --workload $w > "$O/${TAG}_tl_${w}.json" 2>>"$O/${TAG}_tl.err" || { echo "timeline $w rc=$?"; tail -20 "$O/${TAG}_tl.err"; exit 21; }
  python3 -c "
import json; d=json.load(open('$O/${TAG}_tl_${w}.json'))
for k in ('first_after_gap','last_of_25'):
    x=d[k]; print('$w', k, x['ends_us'], x['tiles_per_wave'], x['first_land_us'], x['resolve_start_after_scan_us'], x['rate_tiles_per_us']['all'])"
done
echo done
