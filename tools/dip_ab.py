#!/usr/bin/env python3
"""A/B of scan variants in the driver's own condition: each measurement starts
after the GPU has idled (the shader-clock dip re-arms after a host gap,
DESIGN.md §4.2), then W warm-up + K timed launches back to back, scan time by
HIP events on the launch stream.  Variants (development library, environment
per handle) are interleaved round by round in one process.

    python tools/dip_ab.py "SYNCR_CDC_ABLATE=8" "SYNCR_CDC_ABLATE=12" --rounds 4
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from benchlib import workloads as WL  # noqa: E402

syncr_amd.use_dev_library()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--events", action="store_true",
                    help="time the scan by HIP events bound to its dispatch (kernels without device-clock stamps)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--idle", type=float, default=0.5)
    ap.add_argument("--workload", default="zipf10k", choices=["zipf10k", "uniform1k", "shard8", "shard4", "shard2", "dense", "periodic", "dense1"])
    args = ap.parse_args()
    sizes = WL.zipf_sizes()
    if args.workload == "uniform1k":
        lens, idx = np.full(1024, 1 << 20, np.uint64), np.arange(1024, dtype=np.uint64)
    elif args.workload == "dense1":                # one 128 MiB periodic-64 file
        lens, idx = np.full(1, 128 << 20, np.uint64), np.arange(1, dtype=np.uint64)
    elif args.workload in ("shard8", "shard4", "shard2"):
        sh = WL.lpt_shard(sizes, int(args.workload[5:]))[0]
        lens, idx = sizes[sh], sh.astype(np.uint64)
    else:
        lens, idx = sizes, np.arange(sizes.size, dtype=np.uint64)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    base = syncr_amd.Chunker()
    buf = syncr_amd.DeviceBuffer(base, span)
    buf.gen_corpus(offs, lens, indices=idx)
    if args.workload == "dense":                   # the adversarial table (benchlib.legs.fill_dense)
        from benchlib import legs as LG
        LG.fill_dense(buf, offs, lens, idx)
    elif args.workload in ("periodic", "dense1"):              # the zipf10k table, every byte of the 64-byte period
        pat = WL.periodic_pattern()
        chunk = 256 << 20
        for o in range(0, span, chunk):
            n = min(chunk, span - o)
            buf.upload(np.resize(np.roll(pat, -(o % pat.size)), n), offset=o)
    handles = []
    for v in args.variants:
        saved = dict(os.environ)
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=", 1)
            os.environ[k] = val
        c = syncr_amd.Chunker()
        os.environ.clear()
        os.environ.update(saved)
        c.plan(offs, lens, span)
        c.launch(buf.ptr)
        c.fetch()
        handles.append((v, c))
    res = {v: {"scan": [], "step": []} for v, _ in handles}
    for rnd in range(args.rounds):
        for v, c in (handles if rnd % 2 == 0 else handles[::-1]):     # alternate the order (no first-slot bias)
            c.synchronize()
            time.sleep(args.idle)
            for _ in range(args.warmup):
                c.launch(buf.ptr)
            c.synchronize()
            c.set_timing(True, scan_only=True, events=args.events)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                c.launch(buf.ptr)
            c.synchronize()
            dt = (time.perf_counter() - t0) / args.steps * 1e3
            ms, n = c.kernel_times()
            c.set_timing(False)
            res[v]["scan"].append(ms[0] / n if n else float("nan"))
            res[v]["step"].append(dt)
    out = {"workload": args.workload, "bytes": span, "steps": args.steps, "warmup": args.warmup, "variants": {}}
    for v, _ in handles:
        sc, st = res[v]["scan"], res[v]["step"]
        out["variants"][v] = {"scan_ms_med": round(statistics.median(sc), 4), "scan_ms": [round(x, 4) for x in sc],
                              "step_ms_med": round(statistics.median(st), 4), "step_ms": [round(x, 4) for x in st],
                              "scan_frac_med": round(span / (statistics.median(sc) / 1e3) / 8e12, 4)}
    print(json.dumps(out))
    buf.free()


if __name__ == "__main__":
    main()
