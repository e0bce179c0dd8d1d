#!/bin/bash
# Alternating fresh-process bench runs: warm-up fetch after step 1 (product)
# vs no fetch before the timed region (A/B of the host gap's clock dip).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
for k in 1 2 3; do
  for f in first after; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --sustained-steps 0 --pipeline-depth 1 --no-hashed --no-read-probe --fetch-at $f > $O/gap_$f$k.json 2> $O/gap_$f$k.err || { tail -5 $O/gap_$f$k.err; exit 11; }
    python3 -c "import json,sys; d=json.loads(open('$O/gap_$f$k.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
