#!/bin/bash
# A/B of the split-walk geometry (segment size, worker blocks) on the dense
# workloads, development library, one process per workload.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for w in dense dense1; do
  timeout -k 10 400 python -u tools/ab_bench.py --workload $w --rounds 4 --steps 8 \
    "SYNCR_CDC_SPLIT_SEGC=4096,SYNCR_CDC_SPLIT_BLOCKS=256" "SYNCR_CDC_SPLIT_SEGC=4096,SYNCR_CDC_SPLIT_BLOCKS=512" \
    "SYNCR_CDC_SPLIT_SEGC=2048,SYNCR_CDC_SPLIT_BLOCKS=512" "SYNCR_CDC_SPLIT_SEGC=2048,SYNCR_CDC_SPLIT_BLOCKS=1024" \
    "SYNCR_CDC_SPLIT_SEGC=1024,SYNCR_CDC_SPLIT_BLOCKS=1024" "SYNCR_CDC_SPLIT_SEGC=8192,SYNCR_CDC_SPLIT_BLOCKS=256" \
    > gpurun_out/ab_split_$w.log 2>&1 || { echo "ab $w failed"; tail -20 gpurun_out/ab_split_$w.log; exit 1; }
  echo "== $w"; cat gpurun_out/ab_split_$w.log
done
