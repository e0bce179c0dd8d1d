R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/build/ubench_valu > $R/gpurun_out/ubench_valu.log 2>&1 || exit 5
OUT=$R/gpurun_out/prof_sq
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b1.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b2.log 2>&1 || exit 7
echo ok
