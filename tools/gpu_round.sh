#!/bin/bash
# One GPU-box pass of this round's checks: GPU tests, smoke(), the driver's
# bench command.  Each GPU step has its own time limit; the first failure ends
# the call.
#   bash tools/gpu_round.sh [TAG] [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p "$O"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$O/${TAG}_tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -40 "$O/${TAG}_tests.log"; exit 11; }
tail -3 "$O/${TAG}_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1 || { echo "smoke failed rc=$?"; tail -20 "$O/${TAG}_smoke.log"; exit 12; }
tail -c 600 "$O/${TAG}_smoke.log"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || { echo "bench failed rc=$?"; tail -30 "$O/${TAG}_bench.err"; exit 13; }
python - "$O/${TAG}_bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "hashed", d["hashed"]["value"])
print("parity", json.dumps(d["parity"].get("summary")))
for k in ("uniform1k", "dedup", "dense", "ingest", "ingest_files", "h2d_probe"):
    v = d.get(k) or {}
    print(k, {x: v.get(x) for x in ("value", "ms_per_step", "scan_frac", "frac_of_h2d", "host_stage_seconds", "error")})
s8 = d.get("shard8") or {}
print("shard8", {x: s8.get(x) for x in ("mean_step_frac", "mean_scan_frac", "max_step_ms", "projected_n8_value", "error")})
print("sustained", (d.get("sustained") or {}).get("value"))
print("legs_seconds", d.get("legs_seconds"))
PY
