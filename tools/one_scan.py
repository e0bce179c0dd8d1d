#!/usr/bin/env python3
"""Run one engine variant on the zipf10k corpus for --launches launches (for
rocprofv3 counter passes).  The variant is taken from the environment
(SYNCR_CDC_NB, SYNCR_CDC_MFVAR, SYNCR_CDC_ABLATE, SYNCR_CDC_RUN, ...), read only by
the development library (python -m syncr_amd.build --dev), which this loads.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d out -- python3 tools/one_scan.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402

syncr_amd.use_dev_library()                  # the product library ignores the environment


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--workload", default="zipf10k")
    args = ap.parse_args()
    sizes, idx, _ = bench.workload(args.workload, 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    ch = syncr_amd.Chunker()
    buf = syncr_amd.DeviceBuffer(ch, span)
    buf.gen_corpus(offs, sizes, indices=idx)
    ch.plan(offs, sizes, span)
    for _ in range(args.launches):
        ch.launch(buf.ptr)
    cuts = ch.fetch()
    print("cuts", sum(c.size for c in cuts), "info", ch.info())
    buf.free()


if __name__ == "__main__":
    main()
