#!/usr/bin/env python3
"""One small-batch BASELINE leg through the PRODUCT library, for a kernel
trace (rocprofv3 --kernel-trace -- python3 tools/legs_trace.py ...): exactly
bench.py's leg timing (benchlib/legs.py time_steps: 1 launch + fetch, W-1
launches, K timed launches, 5 phase-timed launches).  tools/legs_trace_show.py
turns the trace into where each timed step's time goes.

    python tools/legs_trace.py --workload uniform1k|shard8|zipf10k|dense|dense1 [--shard R] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from benchlib import legs as L  # noqa: E402
from benchlib import workloads as WL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uniform1k", choices=["uniform1k", "shard8", "zipf10k", "dense", "dense1"])
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--hashed", action="store_true", help="chunk + BLAKE3 (launch_hashed) instead of boundaries only")
    ap.add_argument("--no-events", action="store_true",
                    help="time the K steps with no HIP events at all (what the events cost a small step)")
    args = ap.parse_args()
    sizes = WL.zipf_sizes()
    if args.workload == "uniform1k":
        lens, idx = np.full(1024, 1 << 20, np.uint64), np.arange(1024, dtype=np.uint64)
    elif args.workload == "shard8":
        sh = WL.lpt_shard(sizes, 8)[args.shard]
        lens, idx = sizes[sh], sh.astype(np.uint64)
    elif args.workload == "dense1":                # one 128 MiB periodic-64 file (bench dense1 leg)
        lens, idx = np.full(1, WL.DENSE1_BYTES, np.uint64), np.zeros(1, np.uint64)
    else:                                          # zipf10k / dense: the config-3 file table
        lens, idx = sizes, np.arange(sizes.size, dtype=np.uint64)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    with syncr_amd.Chunker() as ch:
        b = syncr_amd.DeviceBuffer(ch, span)
        try:
            if args.workload == "dense1":
                b.upload(np.resize(WL.periodic_pattern(), span))
            else:
                b.gen_corpus(offs, lens, indices=idx)
                if args.workload == "dense":
                    L.fill_dense(b, offs, lens, idx)
            ch.plan(offs, lens, span)
            if args.no_events:
                import time
                ch.launch(b.ptr)
                ch.fetch()
                for _ in range(args.warmup - 1):
                    ch.launch(b.ptr)
                ch.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    ch.launch(b.ptr)
                ch.synchronize()
                dt = (time.perf_counter() - t0) / args.steps
                r = {"ms_per_step": round(dt * 1e3, 4), "value": round(span / dt / 2**30, 3), "events": False}
            else:
                r = L.time_steps(ch, b.ptr, span, args.steps, args.warmup, hashed=args.hashed)
        finally:
            b.free()
    r.update({"workload": args.workload, "shard": args.shard, "bytes": span, "files": int(lens.size), "hashed": args.hashed,
              "steps": args.steps, "warmup": args.warmup})
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
