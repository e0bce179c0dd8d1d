#!/usr/bin/env python3
"""Scan-time sequence probe: the zipf10k corpus chunked in phases, to see how the
scan kernel's duration depends on what ran before it.  Run under
`rocprofv3 --kernel-trace` and read the per-dispatch durations in order
(tools/scan_seq_show.py), or alone (prints per-phase HIP-event means).

  phase A: 20 plain launches back to back (bench.py's headline region)
  phase B: 5 hashed launches (bench.py's hashed leg)
  phase C: 20 plain launches again
  phase D: 10 plain launches, each after a 2 ms host sleep (GPU idle between)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402

if "--dev" in sys.argv:                  # variants by environment (SYNCR_CDC_ABLATE=5: ROLL2)
    syncr_amd.use_dev_library()


def main():
    sizes, idx, _ = bench.workload("zipf10k", 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    ch = syncr_amd.Chunker()
    buf = syncr_amd.DeviceBuffer(ch, span)
    buf.gen_corpus(offs, sizes, indices=idx)
    ch.plan(offs, sizes, span)
    ch.launch(buf.ptr)
    ch.fetch()

    def phase(name, n, hashed=False, sleep=0.0):
        ch.synchronize()
        ch.set_timing(True, scan_only=not hashed)
        t0 = time.perf_counter()
        for _ in range(n):
            ch.launch(buf.ptr, hashed=hashed)
            if sleep:
                ch.synchronize()
                time.sleep(sleep)
        ch.synchronize()
        dt = (time.perf_counter() - t0) / n
        ms, k = ch.kernel_times()
        ch.set_timing(False)
        print(f"{name}: step {dt * 1e3:.4f} ms  scan {ms[0] / k:.4f} ms ({span / (ms[0] / k) / 1e6:.0f} GB/s)",
              flush=True)

    phase("A plain", 20)
    phase("B hashed", 5, hashed=True)
    phase("C plain", 20)
    phase("D plain+idle", 10, sleep=0.002)
    phase("E plain", 20)
    buf.free()
    ch.close()


if __name__ == "__main__":
    main()
