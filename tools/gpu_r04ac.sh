#!/bin/bash
# Stream tiles with the kept halos (dev SYNCR_CDC_ABLATE=18): the GPU suite with
# it forced (dev library), then A/B against the product stream tiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04ac}
mkdir -p "$O"
SYNCR_TEST_DEV_LIBRARY=1 SYNCR_CDC_ABLATE=18 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not product_ignores and not capi" > "$O/${TAG}_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 10; }
tail -1 "$O/${TAG}_tests.log"
for w in zipf10k shard8; do
  timeout -k 10 240 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=0" "SYNCR_CDC_ABLATE=18" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 11; }
done
cat "$O/${TAG}_dipab.jsonl"
cd /tmp && export TMPDIR=/tmp
SYNCR_CDC_ABLATE=18 timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B TCC_EA0_RDREQ --output-format csv -d $O/prof_${TAG}/pmc_fetch -o run -- python3 $R/tools/one_scan.py > $O/${TAG}_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/${TAG}_pmc.log; exit 12; }
echo done
