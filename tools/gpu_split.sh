# Split walks: parity tests, then dense / dense1 / zipf10k timings (split vs unsplit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { tail -40 gpurun_out/split_tests.log; exit 11; }
tail -3 gpurun_out/split_tests.log
for wl in dense1 dense; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --sustained-steps 0 --no-read-probe > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err || { tail -20 gpurun_out/bench_$wl.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$wl.json')); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], r['kernel_ms'], r['dense_ms'], r['resolve_ms'], d['pipelined'] and d['pipelined']['value'], 'hashed', d['hashed'] and (d['hashed']['value'], d['hashed']['hash_ms']))"
done
timeout -k 10 300 python -u tools/ab_bench.py "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_ABLATE=8,SYNCR_CDC_RESOLVE=nosplit" --rounds 4 > gpurun_out/ab_split.log 2>&1 || { tail -20 gpurun_out/ab_split.log; exit 13; }
cat gpurun_out/ab_split.log
timeout -k 10 300 python -u tools/ab_bench.py "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_ABLATE=8,SYNCR_CDC_RESOLVE=nosplit" --rounds 2 --workload dense > gpurun_out/ab_split_dense.log 2>&1 || { tail -20 gpurun_out/ab_split_dense.log; exit 14; }
cat gpurun_out/ab_split_dense.log
