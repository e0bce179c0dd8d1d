#!/bin/bash
# Round-4 closing pass: GPU tests + smoke + the driver's bench (gpu_round.sh),
# the headline profile (prof.sh), then the dense workload's kernel trace and
# traffic passes and dense1's trace.  First failure ends the call.
#   bash tools/gpu_r04final.sh TAG PROFTAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r04p}
PT=${2:-r04_v1}
bash tools/gpu_round.sh "$TAG" || exit $?
bash tools/prof.sh "$PT" || exit $?
O=$R/gpurun_out
P=$O/prof_${PT}dense
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs --sustained-steps 0 --no-hashed --pipeline-depth 1 --no-read-probe --workload dense > $P/bench_trace.log 2>&1 || { echo "dense trace rc=$?"; exit 21; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B TCC_EA0_RDREQ --output-format csv -d $P/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs --no-hashed --workload dense > $P/bench_fetch.log 2>&1 || { echo "dense pmc rc=$?"; exit 22; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs --no-hashed --workload dense > $P/bench_write.log 2>&1 || { echo "dense pmc write rc=$?"; exit 23; }
P1=$O/prof_${PT}dense1
mkdir -p $P1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P1/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs --sustained-steps 0 --no-hashed --pipeline-depth 1 --no-read-probe --workload dense1 > $P1/bench_trace.log 2>&1 || { echo "dense1 trace rc=$?"; exit 24; }
cd "$R"
grep -h '"metric"' $P/bench_trace.log $P1/bench_trace.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['workload'][:40], d['value'], d['ms_per_step'])"
python3 - $P/trace/run_kernel_stats.csv $P1/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for f in sys.argv[1:]:
    print(f.split('/')[-3])
    for r in csv.DictReader(open(f)):
        print("  %-45s %5s %10.1f us" % (r["Name"].split("(")[0].replace("void ", "")[:45], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
echo done
