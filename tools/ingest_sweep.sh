#!/bin/bash
# Ingest pipeline: copy-free ceiling vs full bytes mode, plus a host memcpy probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
out=$R/gpurun_out/ingest_sweep.log
: > "$out"
for cfg in "256 3 16" "512 3 16"; do
  set -- $cfg
  timeout -k 10 200 python3 -u "$R/tools/ingest_bench.py" --batch-mib $1 --depth $2 --copy-threads $3 --file-gib 0 --no-fill --reps 2 >> "$out" 2>&1 || exit 21
done
timeout -k 10 100 python3 -u -c "
import numpy as np, time, ctypes, sys
sys.path.insert(0, '$R')
import syncr_amd
a = np.random.default_rng(0).integers(0, 256, 1 << 30, dtype=np.uint8)
with syncr_amd.Ingest(batch_bytes=1 << 30, depth=1, copy_threads=16) as g:
    for _ in range(2):
        t = time.perf_counter(); d = g.reserve(a.size); d[:] = a; dt = time.perf_counter() - t; g.commit(0); g.flush()
        print('numpy copy 1 GiB into pinned: %.1f GB/s' % (a.size / dt / 1e9), flush=True)
    for _ in range(2):
        t = time.perf_counter(); g.submit(a, 0); dt = time.perf_counter() - t; g.flush()
        print('pool copy (submit) 1 GiB into pinned: %.1f GB/s' % (a.size / dt / 1e9), flush=True)
" >> "$out" 2>&1 || exit 22
cat "$out"
