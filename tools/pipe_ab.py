#!/usr/bin/env python3
"""Config 4's per-rank batches with two batches in flight (development A/B).

For each shard of zipf10k's 8-way LPT split (and uniform1k), K steps timed
three ways, interleaved over rounds in one process:
  one     one handle, K back-to-back launches (the bench's `shard8` step);
  pipe    two handles (own corpus copy, own stream), step k on handle k % 2,
          scans serialised by the library's per-device event registry (the
          bench's headline `pipelined`);
  free    the same two handles with scans NOT serialised (SYNCR_CDC_SERIAL=0,
          development library): the second scan's waves may take the CUs the
          first scan's last stream tiles free.

    python tools/pipe_ab.py [--workloads shard8,uniform1k] [--steps 20] [--rounds 3]
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
from benchlib import legs as L  # noqa: E402
from benchlib import workloads as WL  # noqa: E402

syncr_amd.use_dev_library()
HBM = 8000.0


def batches(names):
    out = []
    if "shard8" in names:
        sizes = WL.zipf_sizes()
        for r, sh in enumerate(WL.lpt_shard(sizes, 8)):
            out.append((f"shard{r}", sizes[sh], sh.astype(np.uint64)))
    if "uniform1k" in names:
        lens = np.full(1024, 1 << 20, np.uint64)
        out.append(("uniform1k", lens, None))
    for w in ("zipf10k", "dense"):
        if w in names:
            sizes = WL.zipf_sizes()
            out.append((w, sizes, np.arange(sizes.size, dtype=np.uint64)))
    return out


def handle(serial):
    if serial:
        os.environ.pop("SYNCR_CDC_SERIAL", None)
    else:
        os.environ["SYNCR_CDC_SERIAL"] = "0"
    try:
        return syncr_amd.Chunker()
    finally:
        os.environ.pop("SYNCR_CDC_SERIAL", None)


def timed(slots, steps):
    for k in range(4):                                  # warm-up, then K timed
        h, b = slots[k % len(slots)]
        h.launch(b.ptr)
    for h, _ in slots:
        h.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        h, b = slots[k % len(slots)]
        h.launch(b.ptr)
    for h, _ in slots:
        h.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="shard8,uniform1k")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    res = {}
    for name, lens, idx in batches(a.workloads.split(",")):
        offs = WL.offsets_of(lens)
        span = int(lens.sum())
        hs = [handle(True), handle(True), handle(False), handle(False)]
        bufs = []
        for h in hs:
            b = syncr_amd.DeviceBuffer(h, span)
            if idx is None:
                b.gen_corpus(offs, lens)
            else:
                b.gen_corpus(offs, lens, indices=idx)
            if name == "dense":
                L.fill_dense(b, offs, lens, idx)
            h.plan(offs, lens, span)
            h.launch(b.ptr)
            h.fetch()
            bufs.append(b)
        s = list(zip(hs, bufs))
        modes = {"one": s[:1], "pipe": s[:2], "free": s[2:4]}
        ms = {m: [] for m in modes}
        for _ in range(a.rounds):
            for m, sl in modes.items():
                ms[m].append(timed(sl, a.steps) * 1e3)
        # parity of every handle's last launch against the golden digests / fixture
        mism = 0
        for h, _ in s:
            cuts = h.fetch()
            if idx is not None:
                mism += G.check_files("dense" if name == "dense" else "zipf10k", cuts,
                                      idx.astype(np.int64))["mismatches"]
        for b in bufs:
            b.free()
        for h in hs:
            h.close()
        row = {m: round(float(np.median(v)), 4) for m, v in ms.items()}
        row.update({f"{m}_frac": round(span / (v / 1e3) / 1e9 / HBM, 4) for m, v in list(row.items())})
        row["mismatches"] = mism
        res[name] = row
        print(json.dumps({name: row}), flush=True)
    sh = [v for k, v in res.items() if k.startswith("shard")]
    if sh:
        print(json.dumps({"shard8_mean_frac": {m: round(float(np.mean([r[m + "_frac"] for r in sh])), 4)
                                               for m in ("one", "pipe", "free")},
                          "shard8_max_ms": {m: max(r[m] for r in sh) for m in ("one", "pipe", "free")}}))


if __name__ == "__main__":
    main()
