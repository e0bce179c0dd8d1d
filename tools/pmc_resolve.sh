#!/bin/bash
# SQ counters of the resolve kernel on one 128 MiB file (bench.py --workload big1, or $2: dense1 = periodic).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
out=$R/${1:-gpurun_out/pmc_resolve}
WL=${2:-big1}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
            "SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $pass -d "$out/p$i" -o run --output-format csv -- python3 "$R/bench.py" --workload $WL --steps 2 --warmup 1 --no-cpu-baseline > "$out/p$i.log" 2>&1 || exit 20
done
echo pmc done
