#!/bin/bash
# Wave-speed heterogeneity of the scan: per-wave rates by placement (XCC, SE, CU,
# SIMD) for the product scan (dynamic groups), its static stride, the roll alone
# (no DMA) and the DMA alone (no roll).  Dev library, SYNCR_CDC_TRACE timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04b}
mkdir -p "$O"
for v in 0 4 6 3; do
  for w in zipf10k uniform1k; do
    SYNCR_CDC_ABLATE=$v timeout -k 10 120 python -u tools/scan_timeline.py --workload $w > "$O/${TAG}_tl_${w}_a$v.json" 2>>"$O/${TAG}_tl.err" || { echo "timeline $w a$v failed rc=$?"; tail -20 "$O/${TAG}_tl.err"; exit 21; }
  done
done
echo done
