#!/bin/bash
# Strong-scaling rehearsal on ONE GPU: the driver's multi-rank
# command with every rank mapped to device 0 (--device-map), N = 2 and 4.  The
# ranks share one card, so `value` is not a scaling figure; the line checks the
# launcher, the shard plan (load_balance), the per-rank objects and the
# max-over-ranks timing end to end.
#   bash tools/gpu_rehearsal.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-rehearsal}
mkdir -p "$O"
for n in 2 4; do
  map=$(python3 -c "print(','.join(['0']*$n))")
  timeout -k 10 420 python -u bench.py --gpus $n --device-map $map --steps 10 --warmup 3 > "$O/${TAG}_n$n.json" 2> "$O/${TAG}_n$n.err" || { echo "rehearsal n=$n failed rc=$?"; tail -30 "$O/${TAG}_n$n.err"; exit 11; }
  python3 - "$O/${TAG}_n$n.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["n_gpus"], d["scaling"], "value", d["value"], "ms", d["ms_per_step"], "lb", json.dumps(d.get("load_balance")))
PY
done
