#!/usr/bin/env python3
"""Interleaved A/B timing of engine variants in ONE process on ONE device.

Variants are environment settings read by syncr_cdc_open of the DEVELOPMENT
library (libsyncr_cdc_dev.so, `python -m syncr_amd.build --dev`; the product
library reads no environment): SYNCR_CDC_RUN, SYNCR_CDC_ABLATE,
SYNCR_CDC_SCAN_GRID, SYNCR_B3_*, ...  The corpus is
generated once; each round times every variant for --steps launches; the
median scan-kernel time and step time per variant are printed.  Cross-call
comparisons are not trusted (devices and clocks differ between gpurun boxes).

    python tools/ab_bench.py "SYNCR_CDC_RUN=80" "SYNCR_CDC_RUN=144" --rounds 5
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402

syncr_amd.use_dev_library()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--workload", default="zipf10k")
    ap.add_argument("--hashed", action="store_true", help="launch_hashed (BLAKE3 of every chunk)")
    args = ap.parse_args()
    sizes, idx, _ = bench.workload(args.workload, 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    base = syncr_amd.Chunker()
    buf = syncr_amd.DeviceBuffer(base, span)
    buf.gen_corpus(offs, sizes, indices=idx)
    if args.workload == "dense":
        from benchlib import legs
        legs.fill_dense(buf, offs, sizes, idx)
    elif args.workload == "dense1":
        buf.upload(np.resize(bench.periodic_pattern(), span))
    handles = []
    for v in args.variants:
        saved = dict(os.environ)
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=", 1)
            os.environ[k] = val
        c = syncr_amd.Chunker()
        os.environ.clear()
        os.environ.update(saved)
        c.plan(offs, sizes, span)
        c.launch(buf.ptr, hashed=args.hashed)
        ref = c.fetch(hashed=args.hashed)
        if handles:                      # every variant must give the first variant's records
            same = all(np.array_equal(a, b) for a, b in zip(ref, handles[0][3]))
            print(f"{v}: records {'identical to' if same else 'DIFFER from'} {handles[0][0]}", flush=True)
        handles.append((v, c, sum(x.size for x in ref), ref))
    res = {v: ([], [], [], [], []) for v, _, _, _ in handles}
    for _ in range(args.rounds):
        for v, c, _, _ in handles:
            c.synchronize()
            c.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                c.launch(buf.ptr, hashed=args.hashed)
            c.synchronize()
            dt = (time.perf_counter() - t0) / args.steps * 1e3
            ms, n = c.kernel_times()
            c.set_timing(False)
            res[v][0].append(ms[0] / n)
            res[v][1].append(dt)
            res[v][2].append(ms[1] / n)
            res[v][3].append(ms[2] / n)
            res[v][4].append(ms[3] / n)
    for v, c, ncuts, _ in handles:
        sc, st, po, rz, hs = res[v]
        print(f"{v:40s} scan med {statistics.median(sc):.4f} min {min(sc):.4f} ms  "
              f"({span / statistics.median(sc) / 1e6:.0f} GB/s)  step med {statistics.median(st):.4f} ms  "
              f"post {statistics.median(po):.4f} resolve {statistics.median(rz):.4f} ms  "
              + (f"hash {statistics.median(hs):.4f} ms ({span / statistics.median(hs) / 1e6:.0f} GB/s)  "
                 if args.hashed else "") +
              f"cuts {ncuts}  {c.info()['scan_grid']} waves")
    buf.free()


if __name__ == "__main__":
    main()
