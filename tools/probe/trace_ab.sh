#!/bin/bash
# kernel trace of the hashed bench for the old and new builds (one box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for L in old new; do
  so=$R/tools/probe/old.so; [ $L = new ] && so=$R/syncr_amd/libsyncr_cdc.so
  OUT=$R/gpurun_out/tab_$L; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/tools/probe/benchlib.py $so --hashed --steps 10 --warmup 2 --no-cpu-baseline --pipeline-depth 1 > $OUT/log 2>&1 || exit 11
done
echo done
