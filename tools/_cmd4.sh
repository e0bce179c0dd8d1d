timeout -k 10 420 python -m pytest tests -x -q -m "gpu" > gpurun_out/t5_gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t5_gpu_tests.log; tail -4 gpurun_out/t5_gpu_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/_sweep.sh "$1"
