#!/bin/bash
# Ingest parity diagnostics (tools/ingest_repro.py): product library, then the
# development library with the static-stride small-batch scan (ABLATE=4).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
TAG=${1:-r04o}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "back_to_back or alternating or two_handles" > "$O/${TAG}_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/${TAG}_tests.log"; exit 10; }
tail -1 "$O/${TAG}_tests.log"
timeout -k 10 300 python -u tools/ingest_repro.py --passes 3 > "$O/${TAG}_repro_prod.jsonl" 2> "$O/${TAG}_repro.err" || { echo "repro prod rc=$?"; tail -20 "$O/${TAG}_repro.err"; exit 11; }
cat "$O/${TAG}_repro_prod.jsonl" | cut -c1-1500
SYNCR_CDC_ABLATE=4 timeout -k 10 300 python -u tools/ingest_repro.py --passes 3 --dev > "$O/${TAG}_repro_a4.jsonl" 2>> "$O/${TAG}_repro.err" || { echo "repro a4 rc=$?"; tail -20 "$O/${TAG}_repro.err"; exit 12; }
cat "$O/${TAG}_repro_a4.jsonl" | cut -c1-1500
echo done
