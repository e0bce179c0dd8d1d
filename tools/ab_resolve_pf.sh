#!/bin/bash
# A/B of the resolve walk's candidate-window prefetch depth (dev library,
# SYNCR_CDC_RESOLVE_PF) on the adversarial workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
for w in dense dense1; do
  timeout -k 10 300 python -u tools/ab_bench.py SYNCR_CDC_RESOLVE_PF=2 SYNCR_CDC_RESOLVE_PF=4 SYNCR_CDC_RESOLVE_PF=8 --workload $w --rounds 5 > $O/ab_pf_$w.log 2>&1 || { tail -20 $O/ab_pf_$w.log; exit 11; }
  grep -E "scan med|records" $O/ab_pf_$w.log
done
