#!/usr/bin/env python3
"""Ingest parity diagnostics: the zipf10k corpus through syncr_ingest (256 MiB
batches, depth 3, as benchlib.legs.ingest_leg) for several passes; every file
is compared with the device-resident chunking of the same corpus, and each
mismatching file is located in its batch (offset, tile, batch tiles) with its
missing / extra cut ends.

    python tools/ingest_repro.py [--passes 3] [--batch-mib 256] [--depth 3] [--dev]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from benchlib import workloads as WL  # noqa: E402

TILE = 18432


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--batch-mib", type=int, default=256)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--dev", action="store_true")
    args = ap.parse_args()
    if args.dev:
        syncr_amd.use_dev_library()
    sizes = WL.zipf_sizes()
    idx = np.arange(sizes.size, dtype=np.uint64)
    offs = WL.offsets_of(sizes)
    span = int(sizes.sum())
    with syncr_amd.Chunker(device=0) as c:
        buf = syncr_amd.DeviceBuffer(c, span)
        try:
            buf.gen_corpus(offs, sizes, indices=idx)
            c.plan(offs, sizes, span)
            c.launch(buf.ptr)
            ref = c.fetch(hashed=False)
            host = buf.download(span)
        finally:
            buf.free()
    files = [host[int(o): int(o + n)] for o, n in zip(offs.tolist(), sizes.tolist())]
    # the pipeline's batch packing (ingest.cpp room(): seal when used + len > cap)
    cap = args.batch_mib << 20
    where, used, b = [], 0, 0
    bspan = []
    for n in sizes.tolist():
        if used and used + n > cap:
            bspan.append(used)
            b, used = b + 1, 0
        where.append((b, used))
        used += n
    bspan.append(used)
    res = {}

    def on_file(tag, status, a):
        res[tag] = (status, a.copy() if a is not None else None)

    out = {"passes": []}
    with syncr_amd.Ingest(device=0, batch_bytes=cap, depth=args.depth, copy_threads=16, on_file=on_file) as g:
        for p in range(args.passes):
            res.clear()
            for i, f in enumerate(files):
                g.submit(f, i)
            g.flush()
            bad = []
            for i in range(len(files)):
                st, a = res[i]
                got = (a["offset"].astype(np.uint64) + a["len"].astype(np.uint64)) if a is not None else np.zeros(0, np.uint64)
                want = ref[i]["offset"].astype(np.uint64) + ref[i]["len"].astype(np.uint64)
                if st != 0 or got.size != want.size or not np.array_equal(got, want):
                    bb, fo = where[i]
                    miss = np.setdiff1d(want, got)[:8].tolist()
                    extra = np.setdiff1d(got, want)[:8].tolist()
                    bad.append({"file": i, "size": int(sizes[i]), "status": int(st), "batch": bb,
                                "batch_span": bspan[bb], "batch_tiles": (bspan[bb] + TILE - 1) // TILE,
                                "file_off_in_batch": fo, "n_got": int(got.size), "n_want": int(want.size),
                                "missing_ends": miss, "extra_ends": extra,
                                "missing_tiles": [int((fo + e - 1) // TILE) for e in miss],
                                "extra_tiles": [int((fo + e - 1) // TILE) for e in extra]})
            out["passes"].append({"pass": p, "mismatching_files": len(bad), "detail": bad[:6]})
            print(json.dumps(out["passes"][-1]), flush=True)
    out["batches"] = len(bspan)
    print(json.dumps({"batches": len(bspan), "batch_tiles_minmax": [min(bspan) // TILE, max(bspan) // TILE]}))


if __name__ == "__main__":
    main()
