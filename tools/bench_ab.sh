#!/bin/bash
# Alternating whole-bench A/B of development-library variants on one box:
#   bash tools/bench_ab.sh OUTDIR ROUNDS "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_ABLATE=10"
# Each round runs `bench.py --dev-lib` once per variant (fresh process, the
# driver's default command otherwise), so the headline's first-launch clock
# regime is part of what is compared.  Prints value / scan frac per run.
out=$1; rounds=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    tag=$(echo "$v" | tr '=,' '__')
    env $(echo "$v" | tr ',' ' ') timeout -k 10 200 python3 "$R/bench.py" --dev-lib --no-cpu-baseline \
        > "$out/r${r}_${tag}.log" 2>&1 || exit 20
    printf '%s round %s: %s\n' "$v" "$r" "$(grep -o '"value": [0-9.]*' "$out/r${r}_${tag}.log" | head -1)"
  done
done
