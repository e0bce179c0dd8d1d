#!/usr/bin/env python3
"""BLAKE3 lane-task size on one batch (development A/B): the same hashed batch
with 1-leaf and 4-leaf lane tasks forced (SYNCR_B3_LPL, development library),
interleaved over rounds in one process; K hashed steps timed by the wall clock
and the hash phase by HIP events.  The product picks 1 leaf up to
B3_SMALL_SPAN (1 GiB) bytes per launch.

    python tools/lpl_ab.py [--workloads uniform1k,shard8,half] [--steps 10] [--rounds 3]
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
from benchlib import golden as G  # noqa: E402
from benchlib import workloads as WL  # noqa: E402

syncr_amd.use_dev_library()


def batch(name):
    sizes = WL.zipf_sizes()
    if name == "uniform1k":
        return np.full(1024, 1 << 20, np.uint64), None
    if name == "shard8":                           # rank 0 of config 4 at N = 8 (1.22 GiB)
        sh = WL.lpt_shard(sizes, 8)[0]
        return sizes[sh], sh
    if name == "half":                             # zipf10k files up to ~512 MiB
        sh = np.arange(sizes.size)
        k = int(np.searchsorted(np.cumsum(sizes), 512 << 20))
        return sizes[sh[:k]], sh[:k]
    raise SystemExit(f"unknown workload {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="uniform1k,shard8,half")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    for name in a.workloads.split(","):
        lens, idx = batch(name)
        offs = WL.offsets_of(lens)
        span = int(lens.sum())
        hs = {}
        for lpl in ("1", "4"):
            os.environ["SYNCR_B3_LPL"] = lpl
            try:
                h = syncr_amd.Chunker()
            finally:
                os.environ.pop("SYNCR_B3_LPL", None)
            b = syncr_amd.DeviceBuffer(h, span)
            if idx is None:
                b.gen_corpus(offs, lens)
            else:
                b.gen_corpus(offs, lens, indices=idx.astype(np.uint64))
            h.plan(offs, lens, span)
            h.launch(b.ptr, hashed=True)
            h.fetch(hashed=True)
            hs[lpl] = (h, b)
        res = {lpl: {"step": [], "hash": []} for lpl in hs}
        for _ in range(a.rounds):
            for lpl, (h, b) in hs.items():
                for _ in range(3):
                    h.launch(b.ptr, hashed=True)
                h.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    h.launch(b.ptr, hashed=True)
                h.synchronize()
                res[lpl]["step"].append((time.perf_counter() - t0) / a.steps * 1e3)
                h.set_timing(True)
                for _ in range(3):
                    h.launch(b.ptr, hashed=True)
                h.synchronize()
                ms, n = h.kernel_times()
                h.set_timing(False)
                res[lpl]["hash"].append(ms[3] / max(n, 1) if len(ms) > 3 else None)
        mism = 0
        for lpl, (h, b) in hs.items():
            got = h.fetch(hashed=True)
            if idx is not None:
                mism += G.check_files("zipf10k", got, idx.astype(np.int64), hashed=True)["mismatches"]
            b.free()
            h.close()
        print(json.dumps({name: {f"lpl{lpl}": {k: round(float(np.median([x for x in v if x is not None])), 4)
                                               for k, v in r.items()} for lpl, r in res.items()},
                          "bytes": span, "mismatches": mism}), flush=True)


if __name__ == "__main__":
    main()
