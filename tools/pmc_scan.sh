#!/bin/bash
# SQ counters of the scan kernel (plain bench), product and compute-only ablation.
#   bash tools/pmc_scan.sh OUTDIR
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
out=$R/${1:-gpurun_out/pmc_scan}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for ab in 0 2; do
  i=0
  for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
              "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    SYNCR_CDC_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc $pass -d "$out/a${ab}p$i" -o run --output-format csv -- python3 "$R/bench.py" --dev-lib --steps 2 --warmup 1 --no-cpu-baseline > "$out/a${ab}p$i.log" 2>&1 || exit 20
  done
done
echo pmc done
