#!/usr/bin/env python3
"""Is the first-launches slowdown of the scan in the shader
clock or in the memory system?  Run under `rocprofv3 --kernel-trace` and read
the per-dispatch durations in order (tools/dip_show.py).  After a 1 s idle gap
each phase launches N kernels back to back on one stream:

  R1: N torch int64 sums over a 10 GB device tensor (pure streaming read,
      almost no VALU per byte)
  S1: N scans of the zipf10k corpus (syncr_cdc_launch, product library)
  R2, S2: the same again
With --dev (development library) it then runs, each after a 1 s gap, N scans
of three variants: the exact scan (SYNCR_CDC_ABLATE=8), staging only
(DMA + copy-out, no roll: ABLATE=3) and roll only (no DMA: ABLATE=6).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402

DEV = "--dev" in sys.argv
if DEV:
    sys.argv.remove("--dev")
    syncr_amd.use_dev_library()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
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
    x = torch.empty(span // 8, dtype=torch.int64, device="cuda")
    x.random_()
    torch.cuda.synchronize()

    def reads(tag):
        time.sleep(1.0)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        e[0].record()
        for i in range(n):
            x.sum()
            e[i + 1].record()
        torch.cuda.synchronize()
        ms = [e[i].elapsed_time(e[i + 1]) for i in range(n)]
        print(f"{tag} torch-sum ms: " + " ".join(f"{m:.3f}" for m in ms), flush=True)

    def scans(tag):
        ch.synchronize()
        time.sleep(1.0)
        for _ in range(n):
            ch.launch(buf.ptr)
        ch.synchronize()
        print(f"{tag} scans done", flush=True)

    reads("R1")
    scans("S1")
    reads("R2")
    scans("S2")
    if DEV:
        for ab in ("8", "3", "6"):
            os.environ["SYNCR_CDC_ABLATE"] = ab          # read by the dev library at open
            cv = syncr_amd.Chunker()
            cv.plan(offs, sizes, span)
            time.sleep(1.0)
            for _ in range(n):
                cv.launch(buf.ptr)
            cv.synchronize()
            print(f"ABLATE={ab} scans done", flush=True)
            cv.close()
    buf.free()
    ch.close()


if __name__ == "__main__":
    main()
