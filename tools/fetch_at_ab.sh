set -o pipefail
mkdir -p gpurun_out/fa
for r in 1 2 3; do
  for v in end first; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-hashed --sustained-steps 0 --pipeline-depth 1 --no-read-probe --fetch-at $v > gpurun_out/fa/$v.$r.log 2>&1 || exit 1
    python3 -c "import json,sys; l=[x for x in open('gpurun_out/fa/$v.$r.log') if x.startswith('{')][0]; d=json.loads(l); print('$v', $r, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
