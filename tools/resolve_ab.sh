#!/bin/bash
# GPU parity tests, then resolve timing of SYNCR_CDC_RESOLVE variants on big1
# (one 128 MiB file) and zipf10k.  Usage: resolve_ab.sh [variant ...]
# ("default" = unset; default list: default noburst).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/gpu_tests.log"; exit 11; }
tail -2 "$O/gpu_tests.log"
for w in big1 zipf10k; do
  for v in ${@:-default noburst}; do
    if [ $v = default ]; then unset SYNCR_CDC_RESOLVE; else export SYNCR_CDC_RESOLVE=$v; fi
    timeout -k 10 200 python -u bench.py --dev-lib --workload $w --no-cpu-baseline --no-read-probe --pipeline-depth 1 > "$O/ab_${w}_$v.json" 2> "$O/ab_${w}_$v.err" || { echo "bench $w $v failed"; tail -5 "$O/ab_${w}_$v.err"; exit 12; }
    python -c "import json;d=json.load(open('$O/ab_${w}_$v.json'));r=d['roofline'];print('$w $v', d['value'], d['ms_per_step'], r['kernel_ms'], r['resolve_ms'])"
  done
done
unset SYNCR_CDC_RESOLVE
