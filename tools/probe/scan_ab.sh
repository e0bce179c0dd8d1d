#!/bin/bash
# scan parity tests, then the plain bench (and the compute-only ablation) alternating old/new builds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread > gpurun_out/scan_tests.log 2>&1 || { tail -30 gpurun_out/scan_tests.log; exit 1; }
tail -2 gpurun_out/scan_tests.log
for ab in 0 2; do
 for i in 1 2; do
  for L in tools/probe/old.so syncr_amd/libsyncr_cdc_dev.so; do     # ablations: development builds only
    SYNCR_CDC_ABLATE=$ab timeout -k 10 200 python -u tools/probe/benchlib.py $L --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sab.json 2>gpurun_out/sab.err || { tail gpurun_out/sab.err; exit 2; }
    python3 -c "import json;d=json.load(open('gpurun_out/sab.json'));r=d['roofline'];print('ablate $ab', '$L'.split('/')[-1], d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
  done
 done
done
