#!/usr/bin/env python3
"""Cost of the scan-timing HIP events inside a timed step loop: K back-to-back
steps with events around every scan (what bench.py's headline and legs do),
and with none, alternating, after one idle
second each; wall clock per step.

    python tools/event_overhead.py [--workload uniform1k|zipf10k|shard8] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from benchlib import workloads as WL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uniform1k")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    sizes = WL.zipf_sizes()
    if args.workload == "uniform1k":
        lens = np.full(1024, 1 << 20, np.uint64)
        idx = np.arange(1024, dtype=np.uint64)
    elif args.workload == "shard8":
        sh = WL.lpt_shard(sizes, 8)[0]
        lens, idx = sizes[sh], sh.astype(np.uint64)
    else:
        lens, idx = sizes, np.arange(sizes.size, dtype=np.uint64)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    res = {"none": [], "every": []}
    with syncr_amd.Chunker() as c:
        buf = syncr_amd.DeviceBuffer(c, span)
        try:
            buf.gen_corpus(offs, lens, indices=idx)
            c.plan(offs, lens, span)
            c.launch(buf.ptr)
            c.fetch()
            for _ in range(args.rounds):
                for mode in ("none", "every"):
                    time.sleep(1.0)
                    for _ in range(args.warmup):
                        c.launch(buf.ptr)
                    c.synchronize()
                    c.set_timing(mode == "every", scan_only=True)
                    t0 = time.perf_counter()
                    for k in range(args.steps):
                        c.launch(buf.ptr)
                    c.synchronize()
                    dt = (time.perf_counter() - t0) / args.steps
                    c.set_timing(False)
                    res[mode].append(round(dt * 1e3, 4))
        finally:
            buf.free()
    print(json.dumps({"workload": args.workload, "bytes": span, "steps": args.steps, "ms_per_step": res,
                      "median": {k: float(np.median(v)) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
