#!/bin/bash
# GPU hash tests, then the hashed bench alternating old/new libraries on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py -x -v --timeout 120 --timeout-method thread > gpurun_out/hash_tests.log 2>&1 || { tail -30 gpurun_out/hash_tests.log; exit 1; }
tail -3 gpurun_out/hash_tests.log
for i in 1 2; do
  for L in tools/probe/old.so syncr_amd/libsyncr_cdc.so; do
    timeout -k 10 200 python -u tools/probe/benchlib.py $L --hashed --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hab.json 2>gpurun_out/hab.err || { tail gpurun_out/hab.err; exit 2; }
    python3 -c "import json;d=json.load(open('gpurun_out/hab.json'));print('$L', d['value'], d['ms_per_step'], {k:v for k,v in d.items() if k.endswith('_ms')})"
  done
done
