#!/bin/bash
# SQ / HBM counters of the BLAKE3 kernels (bench.py --hashed), one rocprofv3 pass each.
#   bash tools/pmc_hash.sh OUTDIR
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
out=$R/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
            "SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $pass -d "$out/p$i" -o run --output-format csv -- python3 "$R/bench.py" --hashed --steps 2 --warmup 1 --no-cpu-baseline > "$out/p$i.log" 2>&1 || exit 20
done
echo pmc done
