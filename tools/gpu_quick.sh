#!/bin/bash
# Quick GPU pass: a test subset, the bench line without the legs, and the
# dense workload under the kernel trace.   bash tools/gpu_quick.sh TAG "pytest -k expr"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-quick}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" > "$O/${TAG}_tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -40 "$O/${TAG}_tests.log"; exit 11; }
tail -2 "$O/${TAG}_tests.log"
for w in zipf10k dense dense1 uniform1k; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-legs --no-cpu-baseline --no-hashed --sustained-steps 40 > "$O/${TAG}_bench_$w.json" 2> "$O/${TAG}_bench_$w.err" || { echo "bench $w failed"; tail -20 "$O/${TAG}_bench_$w.err"; exit 12; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];s=d['sustained'];print('$w', d['value'], d['ms_per_step'], 'scan', r['kernel_ms'], 'dense', r['dense_ms'], 'resolve', r['resolve_ms'], 'sust', s['value'], s['scan_ms'], 'pipe', d['pipelined']['value'])" "$O/${TAG}_bench_$w.json"
done
for w in dense uniform1k zipf10k; do
bash tools/prof_dense.sh ${TAG}_$w --workload $w > /dev/null && echo "== $w" && python3 - "$O/prof_${TAG}_$w/trace/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
last = {}
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '')
    last.setdefault(n, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for n, v in last.items():
    v = v[-5:]
    print(f"{n[:45]:45s} last5 mean {sum(v)/len(v):9.1f} us")
k = max(i for i, r in enumerate(rows) if 'scan_kernel' in r['Kernel_Name'])
k0 = max(i for i, r in enumerate(rows[:k]) if 'scan_kernel' in r['Kernel_Name'])
t0 = int(rows[k0]['Start_Timestamp'])
for r in rows[k0:k + 1]:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '')
    print(f"   {n[:40]:40s} start {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} end {(int(r['End_Timestamp']) - t0) / 1e3:9.1f}")
PY
done
