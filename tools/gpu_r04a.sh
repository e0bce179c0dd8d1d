#!/bin/bash
# Round 4, first GPU pass: GPU tests + smoke + the driver's bench command
# (tools/gpu_round.sh), then where the small batches' time goes: the dev scan
# timeline (tools/scan_timeline.py) and the product legs under the kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04a}
mkdir -p "$O"
bash tools/gpu_round.sh $TAG || exit $?
for w in uniform1k "shard8 --shard 0" zipf10k; do
  timeout -k 10 120 python -u tools/scan_timeline.py --workload $w >> "$O/${TAG}_timeline.jsonl" 2>>"$O/${TAG}_timeline.err" || { echo "timeline $w failed rc=$?"; tail -20 "$O/${TAG}_timeline.err"; exit 21; }
done
cat "$O/${TAG}_timeline.jsonl"
# energy per byte: the scan without its warm-up / halo (timing-only ablations, dev library), driver's condition
for w in zipf10k uniform1k; do
  timeout -k 10 180 python -u tools/dip_ab.py "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_ABLATE=12" "SYNCR_CDC_ABLATE=13" --workload $w --rounds 4 >> "$O/${TAG}_dipab.jsonl" 2>>"$O/${TAG}_dipab.err" || { echo "dip_ab $w failed rc=$?"; tail -20 "$O/${TAG}_dipab.err"; exit 23; }
done
cat "$O/${TAG}_dipab.jsonl"
cd /tmp && export TMPDIR=/tmp
for w in uniform1k shard8; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_trace_$w" -o run -- python3 "$R/tools/legs_trace.py" --workload $w > "$O/${TAG}_trace_$w.log" 2>&1 || { echo "trace $w failed rc=$?"; tail -20 "$O/${TAG}_trace_$w.log"; exit 22; }
  tail -1 "$O/${TAG}_trace_$w.log"
done
echo done
