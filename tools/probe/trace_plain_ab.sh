#!/bin/bash
# chunking parity tests, then a kernel trace of the plain bench (one batch in flight) for old and new builds
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_mirror.py -x -q --timeout 400 --timeout-method thread > gpurun_out/plain_tests.log 2>&1 || { tail -20 gpurun_out/plain_tests.log; exit 1; }
tail -1 gpurun_out/plain_tests.log
cd /tmp && export TMPDIR=/tmp
for L in old new; do
  so=$R/tools/probe/old.so; [ $L = new ] && so=$R/syncr_amd/libsyncr_cdc.so
  OUT=$R/gpurun_out/tpl_$L; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/tools/probe/benchlib.py $so --steps 10 --warmup 2 --no-cpu-baseline --pipeline-depth 1 > $OUT/log 2>&1 || exit 11
done
echo done
