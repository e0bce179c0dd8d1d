#!/bin/bash
# effective clock (GRBM_GUI_ACTIVE / 8 / duration) of the scan, old vs new build, product and compute-only
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for ab in 0 2; do
 for L in old new; do
  # SYNCR_CDC_ABLATE is read only by development builds (python -m syncr_amd.build --dev)
  so=$R/tools/probe/old.so; [ $L = new ] && so=$R/syncr_amd/libsyncr_cdc_dev.so
  OUT=$R/gpurun_out/clk_${L}_$ab; mkdir -p $OUT
  SYNCR_CDC_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT -o run -- python3 $R/tools/probe/benchlib.py $so --steps 5 --warmup 2 --no-cpu-baseline > $OUT/log 2>&1 || exit 11
 done
done
echo done
