#!/bin/bash
# GPU-box profiling recipe (round 2): kernel trace of the driver's own bench
# command + separate PMC passes (MI355X_MICROARCH.md HBM/rocprofv3 section: one
# counter group per pass, FETCH_SIZE and WRITE_SIZE never together).
#   bash tools/prof.sh r02_vN      then   python tools/pmc_summary.py r02_vN
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
shift
EXTRA="$@"          # extra bench.py flags
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
# 1. the driver's command (`bench.py --gpus 1 --steps 20 --warmup 5`) under the
#    kernel trace: the per-dispatch CSV separates the timed window from the rest
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $EXTRA > $OUT/bench_trace.log 2>&1 || exit 11
# 2./3. HBM bytes per launch (scan and, from the hashed leg, the BLAKE3 leaf).
#    Reads from the request-size counters: gfx950's FETCH_SIZE counts a 128-byte
#    request as 64 B (profiles/r02_fetch_calibration.json, tools/ubench_fetch.hip)
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_32B TCC_EA0_RDREQ --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs $EXTRA > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs $EXTRA > $OUT/bench_write.log 2>&1 || exit 13
# 4. clock and instruction mix of the scan (GRBM_GUI_ACTIVE / 8 XCDs / duration = shader clock)
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --pipeline-depth 1 --sustained-steps 0 --no-read-probe --no-legs $EXTRA > $OUT/bench_sq.log 2>&1 || exit 14
echo done
