#!/bin/bash
# GPU-box profiling recipe (round 1): kernel trace + separate PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
shift
EXTRA="$@"          # extra bench.py flags, e.g. --hashed
# --pipeline-depth 1: profile exactly the timed region (one batch in flight);
# the pipelined segment overlaps launches, so its per-dispatch times differ
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipeline-depth 1 $EXTRA > $OUT/bench_trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 $EXTRA > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 $EXTRA > $OUT/bench_write.log 2>&1 || exit 13
echo done
