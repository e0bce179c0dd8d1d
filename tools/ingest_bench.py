#!/usr/bin/env python3
"""End-to-end rate of the batched ingest pipeline (syncr_ingest_*): host bytes
-> pinned staging -> H2D -> scan + resolve + BLAKE3 -> ChunkInfo per file on
the host, i.e. what a directory walk gets.

  bytes: the zipf10k corpus sits in ordinary host memory
         (as after read()); each file is submit()ted (copied into pinned
         staging by copy_threads host threads)
  files: --file-gib of the corpus written to files under $TMPDIR (page cache
         warm), submit_file()d (pread straight into pinned staging)

A sample of files is checked against the CPU oracle (boundaries + BLAKE3).
Prints one JSON line.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-mib", type=int, default=256)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--copy-threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--file-gib", type=float, default=2.0)
    ap.add_argument("--check-files", type=int, default=200)
    ap.add_argument("--devices", default=None,
                    help="comma-separated device list for syncr_ingest_open_multi (e.g. 0,0 on a one-GPU box); "
                         "default: one device, syncr_ingest_open")
    ap.add_argument("--no-fill", action="store_true",
                    help="diagnostic: reserve/commit without writing the bytes (pipeline ceiling without the "
                         "host copy; results are not checked)")
    args = ap.parse_args()

    sizes, idx, _ = bench.workload("zipf10k", 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    with syncr_amd.Chunker() as ch:                          # corpus bytes, generated once
        dev = syncr_amd.DeviceBuffer(ch, span)
        dev.gen_corpus(offs, sizes, indices=idx)
        host = dev.download(span)
        dev.free()
    files = [host[int(o): int(o + n)] for o, n in zip(offs.tolist(), sizes.tolist())]

    counts = {"chunks": 0, "files": 0}
    keep = {}
    check_ids = set(np.linspace(0, len(files) - 1, min(args.check_files, len(files))).astype(int).tolist())

    def on_file(tag, status, a):
        counts["files"] += 1
        counts["chunks"] += a.size
        if tag in check_ids:
            keep[tag] = a

    devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    out = {"workload": "zipf10k", "bytes": span, "files": len(files), "batch_mib": args.batch_mib,
           "depth": args.depth, "copy_threads": args.copy_threads, "devices": devices}
    with syncr_amd.Ingest(batch_bytes=args.batch_mib << 20, depth=args.depth,
                          copy_threads=args.copy_threads, on_file=on_file, devices=devices) as g:
        best = None
        for _ in range(args.reps):
            counts["files"] = counts["chunks"] = 0
            t0 = time.perf_counter()
            for i, f in enumerate(files):
                if args.no_fill:
                    g.reserve(f.size)
                    g.commit(i)
                else:
                    g.submit(f, i)
            g.flush()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out.update({"bytes_mode_s": round(best, 4), "bytes_mode_GiBps": round(span / best / 2**30, 2),
                    "chunks": counts["chunks"], "no_fill": args.no_fill})
        if args.no_fill:
            print(json.dumps(out), flush=True)
            return
        st = g.stats()
        out["batches_per_pass"] = st["batches"] // args.reps
        if devices:
            out["device_stats"] = g.device_stats()

        # correctness sample vs the oracle (boundaries + BLAKE3)
        from oracle import oracle as O
        bad = 0
        for t in sorted(check_ids):
            f = files[t]
            ends = O.chunk_production(f).astype(np.uint64)
            starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)[:ends.size]
            a = keep[t]
            hs = O.blake3_batch(f, starts, ends - starts, nthreads=8) if ends.size else np.zeros((0, 32), np.uint8)
            bad += not (np.array_equal(a["offset"], starts) and np.array_equal(a["hash"], hs))
        out["sample_checked"] = len(check_ids)
        out["sample_mismatched"] = bad

        # files mode: a prefix of the corpus written under $TMPDIR
        if args.file_gib > 0:
            d = tempfile.mkdtemp(prefix="syncr_ingest_")
            try:
                paths, tot = [], 0
                for i, f in enumerate(files):
                    if tot >= args.file_gib * 2**30:
                        break
                    p = os.path.join(d, f"f{i:05d}")
                    f.tofile(p)
                    paths.append(p)
                    tot += f.size
                best = None
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    for i, p in enumerate(paths):
                        g.submit_file(p, i)
                    g.flush()
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                out.update({"file_mode_files": len(paths), "file_mode_bytes": tot,
                            "file_mode_s": round(best, 4), "file_mode_GiBps": round(tot / best / 2**30, 2)})
            finally:
                shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
