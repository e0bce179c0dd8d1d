#!/bin/bash
# A/B of split-walk geometry (dev library: segment size, worker blocks) on dense1 / dense.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/ab_bench.py SYNCR_CDC_SPLIT_SEGC=4096 SYNCR_CDC_SPLIT_SEGC=1024 SYNCR_CDC_SPLIT_SEGC=2048 SYNCR_CDC_SPLIT_SEGC=8192 SYNCR_CDC_SPLIT_SEGC=2048,SYNCR_CDC_SPLIT_BLOCKS=512 SYNCR_CDC_SPLIT_SEGC=1024,SYNCR_CDC_SPLIT_BLOCKS=512 --workload dense1 --rounds 5 > $O/ab_geom_dense1.log 2>&1 || { tail -20 $O/ab_geom_dense1.log; exit 11; }
grep -E "scan med|DIFFER" $O/ab_geom_dense1.log
timeout -k 10 300 python -u tools/ab_bench.py SYNCR_CDC_SPLIT_SEGC=4096 SYNCR_CDC_SPLIT_SEGC=2048 SYNCR_CDC_SPLIT_SEGC=1024 SYNCR_CDC_SPLIT_SEGC=2048,SYNCR_CDC_SPLIT_BLOCKS=512 --workload dense --rounds 5 > $O/ab_geom_dense.log 2>&1 || { tail -20 $O/ab_geom_dense.log; exit 12; }
grep -E "scan med|DIFFER" $O/ab_geom_dense.log
