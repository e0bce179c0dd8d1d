#!/bin/bash
# SQ stall/issue counters of the scan kernel for a few engine variants.
#   bash tools/pmc_variants.sh OUTDIR "NB=8,MFVAR=3" "NB=8,MFVAR=3,ABLATE=2" ...
# (each variant: comma-separated SYNCR_CDC_* settings without the prefix)
set -e
out=$1; shift
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/$out"
for v in "$@"; do
  tag=$(echo "$v" | tr ',=' '__')
  envs=()
  for kv in $(echo "$v" | tr ',' ' '); do envs+=("SYNCR_CDC_$kv"); done
  for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    p=$(echo $pass | cut -d' ' -f1)
    env "${envs[@]}" timeout -k 10 120 rocprofv3 --pmc $pass -d "$R/$out/$tag/$p" -o run --output-format csv -- python3 "$R/tools/one_scan.py" --launches 2 > "$R/$out/$tag.$p.log" 2>&1
  done
done
