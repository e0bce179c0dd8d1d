#!/bin/bash
# Split-copy kernel A/B (dev SYNCR_CDC_ABLATE=18: 16 waves per record, 16 loads
# in flight per lane, against 8 and 4): split/dense parity on the dev library
# with it forced, then kernel stats of both on dense1 and dense.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04as}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$R"
SYNCR_TEST_DEV_LIBRARY=1 SYNCR_CDC_ABLATE=18 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "not product_ignores and not capi" > "$O/${TAG}_tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 11; }
tail -2 "$O/${TAG}_tests.log"
for w in dense1 dense; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof_$w" -o run -- python3 -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=18" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w failed rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 23; }
done
cat "$O/${TAG}_dipab.jsonl"
find "$O" -name "*kernel_stats.csv" -path "*${TAG}*" -exec grep -H "split_copy" {} \;
echo done
