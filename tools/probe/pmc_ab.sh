#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for L in old new; do
  so=$R/tools/probe/old.so; [ $L = new ] && so=$R/syncr_amd/libsyncr_cdc.so
  OUT=$R/gpurun_out/pab_$L; mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT -o run -- python3 $R/tools/probe/benchlib.py $so --hashed --steps 2 --warmup 1 --no-cpu-baseline > $OUT/log 2>&1 || exit 11
done
echo done
