#!/usr/bin/env python3
"""Golden per-file digests of the full-size benchmark corpora (SURVEY §8d
configs 3 and 5, and the adversarial `dense` workload), computed by the CPU
oracle (oracle/bup_oracle.c, oracle/blake3_oracle.c) on the host-generated
bytes of the same corpora the GPU generates (benchlib/workloads.py).

bench.py's parity leg and the GPU tests compare every file of a GPU run with
these digests, so full-size parity is checked on the driver's box without
running the oracle over 10-32 GiB there.  Fixture contents (npz, no pickles):

  nchunks[i], ends_fnv[i]              production semantics (read_cap 2 MiB,
                                       compute_file_chunks, file_operations.rs:721-788)
  ideal_nchunks[i], ideal_ends_fnv[i]  ideal semantics (chunk_data, tests/chunking_test.rs:170-192)
  hash_fnv[i]                          BLAKE3 of every production chunk
                                       (util::hash_binary, src/util.rs:57-59)

  ends_fnv = FNV-1a-64 over the cut END offsets;
  hash_fnv = FNV-1a-64 over the chunk hashes read as 4 little-endian u64 each.

    python tests/golden/make_corpus_digests.py [zipf10k] [dense] [dense1] [dedup]
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from benchlib import workloads as WL  # noqa: E402
from oracle import oracle as O  # noqa: E402

GOLDEN = os.path.dirname(os.path.abspath(__file__))
NTHR = min(8, os.cpu_count() or 1)


def digests(buf: np.ndarray, offs: np.ndarray, lens: np.ndarray, linear_prod: np.ndarray | None = None) -> dict:
    """Per-file digests of buf's files; linear_prod[i]: use the memmove-free
    production loop for file i (files with millions of chunks)."""
    n = lens.size
    t = time.time()
    lin = np.zeros(n, bool) if linear_prod is None else linear_prod
    prod: list = [None] * n
    for sel, mode in ((np.flatnonzero(~lin), O.MODE_PRODUCTION), (np.flatnonzero(lin), O.MODE_PRODUCTION_WINDOW)):
        if sel.size:
            part = O.chunk_batch(buf, offs[sel], lens[sel], mode=mode, nthreads=NTHR)
            for k, i in enumerate(sel.tolist()):
                prod[i] = part[k]
    print(f"  production: {time.time() - t:.1f} s", flush=True)
    t = time.time()
    ideal = O.chunk_batch(buf, offs, lens, mode=O.MODE_IDEAL, nthreads=NTHR)
    print(f"  ideal: {time.time() - t:.1f} s", flush=True)
    t = time.time()
    co, cn, fi = [], [], []
    for i in range(n):
        e = prod[i].astype(np.uint64)
        s = np.concatenate([[0], e[:-1]]).astype(np.uint64)[:e.size]
        co.append(s + offs[i])
        cn.append(e - s)
    co = np.concatenate(co) if co else np.zeros(0, np.uint64)
    cn = np.concatenate(cn) if cn else np.zeros(0, np.uint64)
    hs = O.blake3_batch(buf, co, cn, nthreads=NTHR)
    print(f"  blake3 of {co.size} chunks: {time.time() - t:.1f} s", flush=True)
    out = {"nchunks": np.array([p.size for p in prod], np.uint32),
           "ends_fnv": np.array([O.fnv_ends(p) for p in prod], np.uint64),
           "ideal_nchunks": np.array([p.size for p in ideal], np.uint32),
           "ideal_ends_fnv": np.array([O.fnv_ends(p) for p in ideal], np.uint64)}
    hf, k = np.zeros(n, np.uint64), 0
    for i in range(n):
        c = prod[i].size
        hf[i] = O.fnv_hashes(hs[k:k + c])
        k += c
    out["hash_fnv"] = hf
    return out


def save(name: str, d: dict, meta: str) -> None:
    path = os.path.join(GOLDEN, f"{name}_digests.npz")
    np.savez_compressed(path, meta=np.array(meta), **d)
    print(f"wrote {path}: {os.path.getsize(path)} bytes, {int(d['nchunks'].sum())} production chunks", flush=True)


def make_zipf10k():
    lens = WL.zipf_sizes()
    t = time.time()
    buf, offs = O.corpus_fill_threads(lens, nthreads=NTHR)
    print(f"zipf10k: {buf.size} bytes generated in {time.time() - t:.1f} s", flush=True)
    save("zipf10k", digests(buf, offs, lens),
         "zipf10k (SURVEY §8d config 3): file i = corpus file i (xorshift64, seed 0x9E3779B97F4A7C15*(i+1), "
         "64 discarded), sizes benchlib.workloads.zipf_sizes(); chunk_bits 20, MAX 16 MiB, read_cap 2 MiB "
         "(production) / unlimited (ideal); oracle/bup_oracle.c + oracle/blake3_oracle.c")


def make_dense():
    lens = WL.zipf_sizes()
    buf, offs = O.corpus_fill_threads(lens, nthreads=NTHR)
    pat = WL.periodic_pattern()
    periodic = np.zeros(lens.size, bool)
    for i in range(lens.size):
        f = WL.dense_file(i, int(lens[i]), pat)
        if f is not None:
            buf[int(offs[i]): int(offs[i] + lens[i])] = f
            periodic[i] = WL.dense_kind(i) == 1
    print(f"dense: {buf.size} bytes, {int(periodic.sum())} periodic files", flush=True)
    save("dense", digests(buf, offs, lens, linear_prod=periodic),
         "dense (adversarial): the zipf10k table, files i%16==5 periodic_pattern() repeated, i%16==11 the "
         "constant byte i&0xff, the rest corpus file i; production cuts of periodic files by the memmove-free "
         "literal loop (orc_chunk_production_window, checked against the literal loop in tests/test_oracle.py)")


def make_dense1():
    n = WL.DENSE1_BYTES
    buf = np.resize(WL.periodic_pattern(), n)
    lens = np.array([n], np.uint64)
    save("dense1", digests(buf, np.zeros(1, np.uint64), lens, linear_prod=np.ones(1, bool)),
         "dense1 (adversarial single file, tests/chunking_test.rs:95-108 / tests/protocol_list_test.rs:360-378 "
         "shape): one DENSE1_BYTES file of periodic_pattern() repeated (an edge every 64 bytes: dense tiles, "
         "millions of chained cuts, split walks); production cuts by orc_chunk_production_window")


def make_dedup():
    plan = WL.dedup_plan()
    base, _ = O.corpus_fill_threads(np.array([WL.DEDUP_BASE], np.uint64), np.array([WL.DEDUP_BASE_INDEX], np.uint64))
    acc = {k: [] for k in ("nchunks", "ends_fnv", "ideal_nchunks", "ideal_ends_fnv", "hash_fnv")}
    step = 64                                             # variants per batch (2 GiB of host memory)
    for b0 in range(0, len(plan), step):
        files = [WL.dedup_file(base, e) for e in plan[b0:b0 + step]]
        lens = np.array([f.size for f in files], np.uint64)
        buf = np.concatenate(files)
        offs = WL.offsets_of(lens)
        d = digests(buf, offs, lens)
        for k in acc:
            acc[k].append(d[k])
        print(f"dedup: {b0 + len(files)} / {len(plan)}", flush=True)
    save("dedup", {k: np.concatenate(v) for k, v in acc.items()},
         "dedup (SURVEY §8d config 5): base = corpus file DEDUP_BASE_INDEX (32 MiB), variant j = "
         "benchlib.workloads.dedup_file(base, dedup_plan()[j])")


if __name__ == "__main__":
    which = sys.argv[1:] or ["zipf10k", "dense", "dense1", "dedup"]
    for w in which:
        {"zipf10k": make_zipf10k, "dense": make_dense, "dense1": make_dense1, "dedup": make_dedup}[w]()
