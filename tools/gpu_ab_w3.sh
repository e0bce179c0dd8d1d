# A/B of the three-waves-per-SIMD scan (SYNCR_CDC_RUN=96) against the product
# scan (dev library): steady timings, roll-only ablations, SQ counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bench.py "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_RUN=96" "SYNCR_CDC_ABLATE=6" "SYNCR_CDC_RUN=96,SYNCR_CDC_ABLATE=6" --rounds 4 > gpurun_out/ab_w3.log 2>&1 || { tail -30 gpurun_out/ab_w3.log; exit 11; }
cat gpurun_out/ab_w3.log
cd /tmp && export TMPDIR=/tmp
for v in "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_RUN=96"; do
  tag=$(echo "$v" | tr ',=' '__')
  env $(echo $v | tr ',' ' ') timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/gpurun_out/pmc_w3/$tag" -o run -- python3 "$R/tools/one_scan.py" --launches 4 > "$R/gpurun_out/pmc_w3_$tag.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_w3_$tag.log"; exit 12; }
done
echo done
