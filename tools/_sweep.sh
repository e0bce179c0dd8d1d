# usage: bash tools/_sweep.sh "RUN:GRID ..."   (GRID 0 = default)
for cfg in $1; do R=${cfg%%:*}; G=${cfg##*:}
  if [ "$G" = "0" ]; then unset SYNCR_CDC_SCAN_GRID; else export SYNCR_CDC_SCAN_GRID=$G; fi
  SYNCR_CDC_RUN=$R timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sw_${R}_${G}.log 2>&1 || { echo "bench $cfg failed"; tail -3 gpurun_out/sw_${R}_${G}.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sw_${R}_${G}.log').read().strip().splitlines()[-1]);r=d['roofline'];e=d['config']['engine'];print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['resolve_ms'], e['scan_grid'], e['scan_blocks_per_cu'], e['compute_units'])"
done
