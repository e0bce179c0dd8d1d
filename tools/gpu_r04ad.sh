#!/bin/bash
# Ingest copy path (pool workers spin before sleeping; parallel copies from 512 KiB):
# the ingest GPU tests, then the ingest bench (tools/ingest_bench.py) and the bench's legs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04ad}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 300 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 10; }
tail -1 "$O/${TAG}_tests.log"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || { echo "bench rc=$?"; tail -20 "$O/${TAG}_bench.err"; exit 11; }
python3 - "$O/${TAG}_bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("ingest", "ingest_files"):
    v = d[k]; print(k, v["value"], v.get("frac_of_h2d"), v.get("host_stage_seconds"), v["parity"]["mismatches"])
print("value", d["value"], "parity", d["parity"]["summary"])
PY
