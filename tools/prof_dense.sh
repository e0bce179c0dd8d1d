#!/bin/bash
# Kernel trace of the adversarial dense workload: per-kernel
# durations of scan / dense / prefix / gather / fix / resolve / split copy.
#   bash tools/prof_dense.sh TAG [extra bench.py flags]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dense}
shift
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs --sustained-steps 0 --no-hashed --pipeline-depth 1 --no-read-probe --workload dense "$@" > $OUT/bench_trace.log 2>&1 || exit 11
find $OUT -name "*kernel_stats.csv" | head -1 | xargs cat
