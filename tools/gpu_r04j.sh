#!/bin/bash
# Dense tail: GPU parity, then kernel traces of the dense and
# dense1 workloads and the read traffic of the dense workload's kernels.
#   bash tools/gpu_r04j.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r04j}
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 11; }
tail -1 "$O/${TAG}_tests.log"
export TMPDIR=/tmp
P=$O/prof_${TAG}dense
mkdir -p $P
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs --sustained-steps 0 --no-hashed --pipeline-depth 1 --no-read-probe --workload dense > $P/bench_trace.log 2>&1 || { echo "dense trace rc=$?"; tail -20 $P/bench_trace.log; exit 12; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B TCC_EA0_RDREQ --output-format csv -d $P/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs --no-hashed --workload dense > $P/bench_fetch.log 2>&1 || { echo "dense pmc rc=$?"; exit 13; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs --no-hashed --workload dense > $P/bench_write.log 2>&1 || { echo "dense pmc write rc=$?"; exit 14; }
PN=$O/prof_${TAG}densenofuse
mkdir -p $PN
SYNCR_CDC_DENSE_FUSE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PN/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs --sustained-steps 0 --no-hashed --pipeline-depth 1 --no-read-probe --workload dense --dev-lib > $PN/bench_trace.log 2>&1 || { echo "dense nofuse trace rc=$?"; tail -20 $PN/bench_trace.log; exit 17; }
P1=$O/prof_${TAG}dense1
mkdir -p $P1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P1/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs --sustained-steps 0 --no-hashed --pipeline-depth 1 --no-read-probe --workload dense1 > $P1/bench_trace.log 2>&1 || { echo "dense1 trace rc=$?"; tail -20 $P1/bench_trace.log; exit 15; }
cd "$R"
grep -h '"metric"' $P/bench_trace.log $PN/bench_trace.log $P1/bench_trace.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['workload'][:40], d['value'], d['ms_per_step'], d.get('scan_frac'))"
python3 - $P/trace/run_kernel_stats.csv $PN/trace/run_kernel_stats.csv $P1/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for f in sys.argv[1:]:
    print(f.split('/')[-3])
    for r in csv.DictReader(open(f)):
        print("  %-45s %5s %10.1f us" % (r["Name"].split("(")[0].replace("void ", "")[:45], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
timeout -k 10 120 python -u tools/scan_timeline.py --workload dense1 > "$O/${TAG}_tl_dense1.json" 2>"$O/${TAG}_tl.err" || { echo "timeline rc=$?"; tail -20 "$O/${TAG}_tl.err"; exit 16; }
python3 -c "
import json; d=json.load(open('$O/${TAG}_tl_dense1.json'))
for k in ('first_after_gap','last_of_25'):
    x=d[k]; print(k, x['ends_us'], x['tiles_per_wave'], x['tile_us'], x['first_land_us'], x['resolve_start_after_scan_us'])"
echo done
