"""GPU legs of bench.py outside its timed headline region, and of smoke():
parity of the product HIP path against committed golden fixtures and the CPU
oracle, and the single-GPU BASELINE configs other than the headline.

Every leg runs the product library (syncr_amd -> libsyncr_cdc.so); the oracle
(oracle/) is only the checker, exactly as in bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

from benchlib import golden as G
from benchlib import workloads as WL

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
M = 1 << 20


def _tests_path():
    t = os.path.join(G.ROOT, "tests")
    if t not in sys.path:
        sys.path.insert(0, t)


def time_steps(ch, ptr: int, span: int, steps: int, warmup: int, hashed: bool = False) -> dict:
    """K one-in-flight steps after W warm-up steps (results fetched after the
    first), wall clock bracketed by device synchronisation; the scan kernel's
    mean time by the device clock (no queue packets in the timed steps); then a
    few steps with every phase bracketed by events (outside the timed steps)."""
    ch.launch(ptr, hashed=hashed)
    ch.fetch(hashed=hashed)
    for _ in range(max(warmup - 1, 0)):
        ch.launch(ptr, hashed=hashed)
    ch.synchronize()
    ch.set_timing(True, scan_only=True)
    t0 = time.perf_counter()
    for _ in range(steps):
        ch.launch(ptr, hashed=hashed)
    ch.synchronize()
    dt = (time.perf_counter() - t0) / max(steps, 1)
    kms, nl = ch.kernel_times()
    ch.set_timing(False)
    scan = ch.last_scan()                     # the library's report of the scan the timed steps ran
    ch.set_timing(True)
    for _ in range(min(steps, 5)):
        ch.launch(ptr, hashed=hashed)
    ch.synchronize()
    pms, pn = ch.kernel_times()
    ch.set_timing(False)
    scan_ms = kms[0] / max(nl, 1)
    out = {"value": round(span / dt / 2**30, 3), "unit": "GiB/s", "ms_per_step": round(dt * 1e3, 4),
           "scan_ms": round(scan_ms, 4),
           "scan_frac": round(span / (scan_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if scan_ms > 0 else None,
           "dense_ms": round(pms[1] / max(pn, 1), 4), "resolve_ms": round(pms[2] / max(pn, 1), 4),
           "scan_kernel": scan["kernel"], "scan_schedule": scan["kind"]}
    if hashed:
        out["hash_ms"] = round(pms[3] / max(pn, 1), 4)
    return out


def time_pipelined(slots, span: int, steps: int, warmup: int) -> dict:
    """The same K steps with two batches in flight: step k on slot k % 2, each
    slot its own handle, stream and copy of the batch (how the ingest pipeline
    runs its slots; the scans of two handles are not ordered, so the next
    batch's scan takes the CUs the last one's final stream tiles free)."""
    for k in range(max(warmup, 2)):
        h, b = slots[k % 2]
        h.launch(b.ptr)
    for h, _ in slots:
        h.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        h, b = slots[k % 2]
        h.launch(b.ptr)
    for h, _ in slots:
        h.synchronize()
    dt = (time.perf_counter() - t0) / max(steps, 1)
    return {"ms_per_step": round(dt * 1e3, 4),
            "step_frac": round(span / dt / 1e9 / HBM_PEAK_GBS, 4), "value": round(span / dt / 2**30, 3)}


PIPE_NOTE = ("two batches in flight: step k on slot k % 2, each slot its own handle, HIP stream and copy of the "
             "batch (the ingest pipeline's slots); not the one-in-flight step above")


# --------------------------------------------------------------------------
# parity legs against fixtures / the oracle (small inputs)
# --------------------------------------------------------------------------
def kat_leg(device: int = 0) -> dict:
    """Every case of tests/golden/kat_cases.json (SURVEY App. A known answers,
    tests/chunking_test.rs inputs, random data at bits 8..24 and read caps, and
    the adversarial inputs where skipping the chunk-head fix-up changes the cuts
    -- a fresh Bup per chunk, file_operations.rs:748) through the product's
    host entry point, cut ends compared with the fixture; each case's chunks
    are also hashed on the GPU and checked against the BLAKE3 oracle."""
    import syncr_amd
    from oracle import oracle as O
    _tests_path()
    from golden_inputs import make_input
    cases = G.load_json("kat_cases.json")["cases"]
    handles: dict = {}
    bad, hbad, nhash, names = 0, 0, 0, []
    try:
        for c in cases:
            key = (c["chunk_bits"], c["max_chunk"], c["read_cap"])
            if key not in handles:
                handles[key] = syncr_amd.Chunker(*key, device=device)
            ch = handles[key]
            data = make_input(c["recipe"])
            got = ch.batch_arrays(data, [0], [data.size], hashed=True)[0]
            if G.ends_of(got).tolist() != list(c["ends"]):
                bad += 1
                names.append(c["name"])
            if data.size <= 8 * M:
                nhash += got.size
                want = O.blake3_batch(data, got["offset"].astype(np.uint64), got["len"].astype(np.uint64),
                                      nthreads=8) if got.size else np.zeros((0, 32), np.uint8)
                hbad += int((got["hash"] != want).any(axis=1).sum()) if got.size else 0
    finally:
        for h in handles.values():
            h.close()
    out = {"cases": len(cases), "adversarial_head_cases": sum(c["name"].startswith("adversarial_head")
                                                              for c in cases),
           "adversarial_head_b20_cases": sum(c["name"].startswith("adversarial_head_b20") for c in cases),
           "mismatches": bad, "chunk_hashes_checked": nhash, "hash_mismatches": hbad,
           "fixture": "tests/golden/kat_cases.json"}
    if names:
        out["failed"] = names[:8]
    return out


def blake3_vectors_leg(device: int = 0) -> dict:
    """The official BLAKE3 vectors (tests/golden/blake3_vectors.json), each input
    one chunk (chunk_bits 31, no read cap), hashed by the product's GPU hasher."""
    import syncr_amd
    v = G.load_json("blake3_vectors.json")
    lens = np.array([n for n, _ in v["cases"]], np.uint64)
    offs = np.zeros_like(lens)
    pos = 0
    for i, n in enumerate(lens.tolist()):
        offs[i] = pos
        pos += n + 13                           # unaligned file starts
    buf = np.zeros(max(pos, 1), np.uint8)
    for o, n in zip(offs.tolist(), lens.tolist()):
        buf[o:o + n] = (np.arange(n) % 251).astype(np.uint8)
    with syncr_amd.Chunker(31, 1 << 31, 0, device=device) as ch:
        got = ch.batch_arrays(buf, offs, lens, hashed=True)
    bad = 0
    for (n, want), cuts in zip(v["cases"], got):
        if n == 0:
            bad += cuts.size != 0
        else:
            bad += not (cuts.size == 1 and cuts["hash"][0].tobytes().hex() == want)
    return {"cases": len(v["cases"]), "mismatches": bad, "fixture": "tests/golden/blake3_vectors.json"}


def dense_subset_files() -> list[np.ndarray]:
    """Adversarial files after the reference's own test data: constant bytes
    (tests/chunking_test.rs:95-108; 50 MiB of 'A' and 100 000 x 'X',
    tests/protocol_list_test.rs:360-400, scaled), and 64-byte periodic data
    (a candidate every 64 bytes: dense scan tiles, chained cuts, and files
    long enough to be walked split)."""
    pat = WL.periodic_pattern()
    rng = np.random.default_rng(77)
    glitchy = np.resize(pat, 6 * M + 5)
    for g in rng.integers(0, glitchy.size - 4096, 8).tolist():
        glitchy[g: g + int(rng.integers(1, 3000))] = rng.integers(0, 256, 1, dtype=np.uint8)
    return [np.resize(pat, 5 * M + 3), np.full(5 * M, ord("A"), np.uint8), np.resize(pat, 2 * M),
            np.full(100000, ord("X"), np.uint8), glitchy, np.resize(pat, 700 * 1024 + 11),
            np.full(20 * M + 7, 0xAB, np.uint8), rng.integers(0, 256, 3 * M, dtype=np.uint8),
            np.resize(pat, 64 * 1024), np.resize(np.roll(pat, 17), 4 * M + 1)]


def dense_subset_leg(device: int = 0) -> dict:
    """dense_subset_files() through the product path in both semantics, each
    twice (the second launch walks long files split, once the first fetch has
    seen their candidate density), against the oracle."""
    import syncr_amd
    from oracle import oracle as O
    files = dense_subset_files()
    lens = np.array([f.size for f in files], np.uint64)
    offs = WL.offsets_of(lens)
    buf = np.concatenate(files)
    out = {"files": len(files), "bytes": int(lens.sum())}
    bad = 0
    for sem, cap in (("production", syncr_amd.TOKIO_READ_CAP), ("ideal", 0)):
        want = [(O.chunk_production_window(f) if cap else O.chunk_ideal(f)).tolist() for f in files]
        with syncr_amd.Chunker(read_cap=cap, device=device) as ch:
            for rep in range(2):
                got = ch.batch_arrays(buf, offs, lens)
                bad += sum(G.ends_of(g).tolist() != w for g, w in zip(got, want))
            out[f"{sem}_chunks"] = int(sum(g.size for g in got))
            out[f"{sem}_dense_tiles"] = int(ch.last_stats()["dense_tiles"])
            out[f"{sem}_split"] = ch.split_stats()
    out["mismatches"] = bad
    out["checked"] = "oracle (literal loops; orc_chunk_production_window for production), both semantics, 2 launches each"
    return out


# --------------------------------------------------------------------------
# single-GPU BASELINE configs beside the headline (each with its parity)
# --------------------------------------------------------------------------
def uniform1k_leg(device: int, steps: int, warmup: int) -> dict:
    """1024 x 1 MiB files generated in HBM, one batch;
    parity: the committed full cut lists (tests/golden/corpus_uniform_1024x1MiB.json)."""
    import syncr_amd
    g = G.load_json("corpus_uniform_1024x1MiB.json")
    lens = np.full(int(g["files"]), int(g["file_len"]), np.uint64)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    with syncr_amd.Chunker(device=device) as ch, syncr_amd.Chunker(device=device) as ch2:
        b = syncr_amd.DeviceBuffer(ch, span)
        b2 = syncr_amd.DeviceBuffer(ch2, span)
        try:
            b.gen_corpus(offs, lens)
            b2.gen_corpus(offs, lens)
            ch.plan(offs, lens, span)
            ch2.plan(offs, lens, span)
            out = time_steps(ch, b.ptr, span, steps, warmup)
            cuts = ch.fetch()
            ch2.launch(b2.ptr)
            ch2.fetch()
            out["pipelined"] = dict(time_pipelined([(ch, b), (ch2, b2)], span, steps, warmup), note=PIPE_NOTE)
            cuts2 = ch2.fetch()
        finally:
            b.free()
            b2.free()
    bad = sum(G.ends_of(c).tolist() != e for c, e in zip(cuts, g["ends"]))
    bad += sum(G.ends_of(c).tolist() != e for c, e in zip(cuts2, g["ends"]))
    out.update({"config": "SURVEY §8d config 2: 1024 x 1 MiB random files, 1 GiB, production semantics",
                "parity": {"files": len(cuts), "chunks": int(sum(c.size for c in cuts)), "mismatches": int(bad),
                           "fixture": "tests/golden/corpus_uniform_1024x1MiB.json (every cut)"}})
    return out


def shard_leg(device: int, steps: int, warmup: int, nshards: int = 8) -> dict:
    """BASELINE config 4's per-rank work on this one GPU: zipf10k LPT-sharded
    per file into `nshards` shards (exactly what bench.py --gpus N --scaling
    strong gives each rank), each shard generated in HBM and timed as its own
    planned batch (W warm-up + K one-in-flight steps), one shard after another.
    Every shard's files are checked against the golden digests.  The projected
    N-GPU aggregate is the corpus bytes / the slowest shard's step: a one-GPU
    projection, not a measured scaling point (files are independent,
    file_operations.rs:599-605,721-788, so ranks share nothing but the clock)."""
    import syncr_amd
    sizes = WL.zipf_sizes()
    shards = WL.lpt_shard(sizes, nshards)
    biggest = max(int(sizes[s].sum()) for s in shards)
    per, mism, nfiles = [], 0, 0
    with syncr_amd.Chunker(device=device) as ch, syncr_amd.Chunker(device=device) as ch2:
        b = syncr_amd.DeviceBuffer(ch, biggest)
        b2 = syncr_amd.DeviceBuffer(ch2, biggest)
        try:
            for r, sh in enumerate(shards):
                lens = sizes[sh]
                offs = WL.offsets_of(lens)
                span = int(lens.sum())
                b.gen_corpus(offs, lens, indices=sh.astype(np.uint64))
                ch.plan(offs, lens, span)
                t = time_steps(ch, b.ptr, span, steps, warmup)
                p = G.check_files("zipf10k", ch.fetch(), sh)
                # the same shard with two batches in flight
                b2.gen_corpus(offs, lens, indices=sh.astype(np.uint64))
                ch2.plan(offs, lens, span)
                ch2.launch(b2.ptr)
                ch2.fetch()
                tp = time_pipelined([(ch, b), (ch2, b2)], span, steps, warmup)
                p2 = G.check_files("zipf10k", ch2.fetch(), sh)
                mism += p["mismatches"] + p2["mismatches"]
                nfiles += p["files"]
                per.append({"shard": r, "files": int(sh.size), "bytes": span, "ms_per_step": t["ms_per_step"],
                            "scan_ms": t["scan_ms"], "scan_frac": t["scan_frac"],
                            "step_frac": round(span / (t["ms_per_step"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                            "dense_ms": t["dense_ms"], "resolve_ms": t["resolve_ms"],
                            "scan_schedule": t["scan_schedule"], "parity_mismatches": p["mismatches"],
                            "pipelined_ms_per_step": tp["ms_per_step"], "pipelined_step_frac": tp["step_frac"]})
        finally:
            b.free()
            b2.free()
    total = int(sizes.sum())
    worst = max(x["ms_per_step"] for x in per)
    return {"nshards": nshards, "shards": per, "total_bytes": total,
            "max_ms_per_step": worst,
            "projected_value": round(total / (worst / 1e3) / 2**30, 3), "unit": "GiB/s",
            "projected_note": (f"one-GPU projection of the N={nshards} strong-scaling aggregate (BASELINE config 4): "
                               "corpus bytes / the slowest shard's step, each shard timed alone on this GPU; no "
                               "multi-GPU scaling was measured"),
            "mean_step_frac": round(sum(x["step_frac"] for x in per) / len(per), 4),
            "pipelined": {"mean_step_frac": round(sum(x["pipelined_step_frac"] for x in per) / len(per), 4),
                          "max_ms_per_step": max(x["pipelined_ms_per_step"] for x in per),
                          "projected_value": round(total / (max(x["pipelined_ms_per_step"] for x in per) / 1e3)
                                                   / 2**30, 3),
                          "note": PIPE_NOTE},
            "mean_scan_frac": round(sum(x["scan_frac"] for x in per) / len(per), 4),
            "load_balance_max_over_mean_ms": round(worst / (sum(x["ms_per_step"] for x in per) / len(per)), 4),
            "parity": {"files": nfiles, "mismatches": mism, "fixture": "tests/golden/zipf10k_digests.npz",
                       "semantics": "production"}}


def h2d_probe(device: int, nbytes: int = 256 << 20, reps: int = 10) -> dict:
    """The end-to-end path's link ceiling: pinned host memory -> device with
    hipMemcpyAsync (syncr_cdc_memcpy_h2d on the handle's stream), `reps` copies
    of `nbytes`, each timed by the host around a stream synchronisation; and
    the same device -> pinned host."""
    import ctypes
    import syncr_amd
    L = syncr_amd.library()
    out = {}
    with syncr_amd.Chunker(device=device) as ch:
        hp = ctypes.c_void_p()
        syncr_amd._check(L.syncr_cdc_host_alloc_pinned(ch.handle, nbytes, ctypes.byref(hp)), "host_alloc_pinned")
        d = syncr_amd.DeviceBuffer(ch, nbytes)
        try:
            ctypes.memset(hp, 0x5A, nbytes)
            for name, fn, dst, src in (("h2d", L.syncr_cdc_memcpy_h2d, d.ptr, hp.value),
                                       ("d2h", L.syncr_cdc_memcpy_d2h, hp.value, d.ptr)):
                ts = []
                for _ in range(reps + 1):
                    t0 = time.perf_counter()
                    syncr_amd._check(fn(ch.handle, dst, src, nbytes, None), name)
                    ch.synchronize()
                    ts.append(time.perf_counter() - t0)
                ts = ts[1:]                                       # the first copy maps the pages
                out[name] = {"best_gbs": round(nbytes / min(ts) / 1e9, 2),
                             "mean_gbs": round(nbytes / (sum(ts) / len(ts)) / 1e9, 2)}
        finally:
            d.free()
            L.syncr_cdc_host_free_pinned(ch.handle, hp)
    out.update({"bytes_per_copy": nbytes, "copies": reps,
                "path": "hipHostMalloc'd (pinned) buffer <-> device, hipMemcpyAsync on one stream, host-timed per copy"})
    return out


def build_dedup(ch, dbuf, offs, plan) -> None:
    """The dedup corpus on the device: the base is corpus file DEDUP_BASE_INDEX
    (syncr_cdc_gen_corpus), each variant is copied together from base pieces and
    its edit's bytes (syncr_cdc_memcpy_d2d): no 32 GiB host upload."""
    import syncr_amd
    base = syncr_amd.DeviceBuffer(ch, WL.DEDUP_BASE)
    ins_all = np.concatenate([e[3] for e in plan])
    ins_off = WL.offsets_of(np.array([e[3].size for e in plan], np.uint64))
    ins = syncr_amd.DeviceBuffer(ch, max(int(ins_all.size), 16))
    try:
        base.gen_corpus(np.zeros(1, np.uint64), np.array([WL.DEDUP_BASE], np.uint64),
                        indices=np.array([WL.DEDUP_BASE_INDEX], np.uint64))
        ins.upload(ins_all)
        for j, e in enumerate(plan):
            dst = int(offs[j])
            for src, o, n in WL.dedup_pieces(e):
                sp = base.ptr + o if src == "base" else ins.ptr + int(ins_off[j]) + o
                dbuf.copy_from(sp, n, dst)
                dst += n
        ch.synchronize()
    finally:
        base.free()
        ins.free()


def dedup_stability(cuts, plan) -> dict:
    """Share of the base file's cut offsets each variant keeps (offsets past the
    edit shifted back), and a chunk-level dedup ratio."""
    from oracle import oracle as O
    base, _ = O.corpus_fill_threads(np.array([WL.DEDUP_BASE], np.uint64), np.array([WL.DEDUP_BASE_INDEX], np.uint64))
    base_cuts = set(O.chunk_production(base).astype(np.int64).tolist())
    kept = []
    for c, e in zip(cuts, plan):
        pos, delta = e[1], WL.dedup_shift(e)
        ends = G.ends_of(c).astype(np.int64).tolist()
        adj = {x - delta if x > pos else x for x in ends}
        kept.append(len(adj & base_cuts) / max(len(base_cuts), 1))
    return {"base_cuts": len(base_cuts), "kept_median": round(float(np.median(kept)), 4),
            "kept_min": round(float(np.min(kept)), 4),
            "note": "share of the base file's cut offsets present in each variant (offsets past the edit shifted back)"}


def dedup_leg(device: int, steps: int, warmup: int) -> dict:
    """SURVEY §8d config 5 (~32 GiB, one batch), built on the device; parity of
    every variant's cuts and chunk hashes against the golden digests
    (tests/golden/dedup_digests.npz), boundary stability."""
    import syncr_amd
    plan = WL.dedup_plan()
    lens = np.array([e[4] for e in plan], np.uint64)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    with syncr_amd.Chunker(device=device) as ch:
        b = syncr_amd.DeviceBuffer(ch, span)
        try:
            t0 = time.perf_counter()
            build_dedup(ch, b, offs, plan)
            t_build = time.perf_counter() - t0
            ch.plan(offs, lens, span)
            out = time_steps(ch, b.ptr, span, steps, warmup)
            cuts = ch.fetch()
            ch.launch(b.ptr, hashed=True)
            hcuts = ch.fetch(hashed=True)
        finally:
            b.free()
    rows = np.arange(len(plan))
    out.update({"config": "SURVEY §8d config 5: 1000 single-edit variants of one 32 MiB random base "
                          f"({span / 2**30:.2f} GiB), production semantics; built in HBM in {t_build:.2f} s",
                "parity": G.check_files("dedup", cuts, rows),
                "parity_hashed": G.check_files("dedup", hcuts, rows, hashed=True),
                "stability": dedup_stability(cuts, plan)})
    return out


def fill_dense(dbuf, offs, lens, idx) -> None:
    """Overwrite the adversarial files of the dense workload (WL.dense_kind)."""
    pat = WL.periodic_pattern()
    for j in range(lens.size):
        f = WL.dense_file(int(idx[j]), int(lens[j]), pat)
        if f is not None and f.size:
            dbuf.upload(f, offset=int(offs[j]))


def dense_leg(device: int, steps: int, warmup: int) -> dict:
    """The adversarial `dense` workload (zipf10k table; periodic files i%16==5,
    constant files i%16==11) as one batch; parity of every file (cuts and chunk
    hashes) against tests/golden/dense_digests.npz."""
    import syncr_amd
    lens = WL.zipf_sizes()
    idx = np.arange(lens.size, dtype=np.uint64)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    with syncr_amd.Chunker(device=device) as ch:
        b = syncr_amd.DeviceBuffer(ch, span)
        try:
            b.gen_corpus(offs, lens, indices=idx)
            fill_dense(b, offs, lens, idx)
            ch.plan(offs, lens, span)
            out = time_steps(ch, b.ptr, span, steps, warmup)
            cuts = ch.fetch()
            out["split"] = ch.split_stats()
            out["dense_tiles"] = int(ch.last_stats()["dense_tiles"])
            out["candidates"] = int(ch.last_stats()["candidates"])
            hashed = time_steps(ch, b.ptr, span, max(steps // 2, 3), 2, hashed=True)
            hcuts = ch.fetch(hashed=True)
        finally:
            b.free()
    kinds = np.array([WL.dense_kind(int(i)) for i in idx.tolist()])
    out.update({"config": "adversarial: zipf10k table, periodic-64 files (i%16==5) and constant files (i%16==11)",
                "adversarial_bytes_frac": {"periodic64": round(float(lens[kinds == 1].sum()) / span, 4),
                                           "constant": round(float(lens[kinds == 2].sum()) / span, 4)},
                "hashed": {k: hashed[k] for k in ("value", "ms_per_step", "hash_ms")},
                "parity": G.check_files("dense", cuts, idx),
                "parity_hashed": G.check_files("dense", hcuts, idx, hashed=True)})
    return out


def dense1_leg(device: int, steps: int, warmup: int) -> dict:
    """The adversarial single file: one DENSE1_BYTES (128 MiB) file of the
    64-byte period that hits every 64 bytes (the shape of the reference's
    constant-data tests, tests/chunking_test.rs:95-108 and
    tests/protocol_list_test.rs:360-378, with an edge in every period): 2 M
    chained cuts, dense tiles everywhere, split resolve walks.  Timed like the
    other legs (boundaries; then with BLAKE3); parity of its cuts (both
    semantics) and hashes against tests/golden/dense1_digests.npz."""
    import syncr_amd
    span = WL.DENSE1_BYTES
    lens, offs, idx = np.array([span], np.uint64), np.zeros(1, np.uint64), np.zeros(1, np.uint64)
    data = np.resize(WL.periodic_pattern(), span)
    with syncr_amd.Chunker(device=device) as ch, syncr_amd.Chunker(read_cap=0, device=device) as chi:
        b = syncr_amd.DeviceBuffer(ch, span)
        try:
            b.upload(data)
            ch.plan(offs, lens, span)
            out = time_steps(ch, b.ptr, span, steps, warmup)
            cuts = ch.fetch()
            out["split"] = ch.split_stats()
            out["dense_tiles"] = int(ch.last_stats()["dense_tiles"])
            hashed = time_steps(ch, b.ptr, span, max(steps // 2, 3), 2, hashed=True)
            hcuts = ch.fetch(hashed=True)
            chi.plan(offs, lens, span)
            chi.launch(b.ptr)
            icuts = chi.fetch()
        finally:
            b.free()
    out.update({"config": f"adversarial single file: {span} bytes of the periodic-64 pattern",
                "chunks": int(cuts[0].size),
                "step_frac": round(span / (out["ms_per_step"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "hashed": {k: hashed[k] for k in ("value", "ms_per_step", "hash_ms")},
                "parity": G.check_files("dense1", cuts, idx),
                "parity_ideal": G.check_files("dense1", icuts, idx, semantics="ideal"),
                "parity_hashed": G.check_files("dense1", hcuts, idx, hashed=True)})
    return out


def ideal_leg(dbuf, offs, lens, idx, device: int) -> dict:
    """Ideal semantics (chunk_data, tests/chunking_test.rs:170-192: read_cap 0)
    on the headline corpus already in HBM, every file against the golden ideal
    digests."""
    import syncr_amd
    with syncr_amd.Chunker(read_cap=0, device=device) as ch:
        ch.plan(offs, lens, int(lens.sum()))
        ch.launch(dbuf.ptr)
        cuts = ch.fetch()
    return G.check_files("zipf10k", cuts, idx, semantics="ideal")


def ingest_multi_device_leg(host: np.ndarray, offs, lens, idx, device: int, multi_files: int = 2000) -> dict:
    """The multi-device front end (syncr_ingest_open_multi, devices {d, d}) on
    the first `multi_files` zipf10k files from host memory, every file's cuts and
    hashes against the golden digests (a parity leg: the timed end-to-end legs
    are driven from C++, benchlib/e2e.py)."""
    import syncr_amd
    nm = min(multi_files, int(lens.size))
    res: dict = {}
    with syncr_amd.Ingest(devices=[device, device], batch_bytes=64 << 20, depth=2, copy_threads=8,
                          on_file=lambda t, st, a: res.__setitem__(t, a)) as g:
        for i in range(nm):
            g.submit(host[int(offs[i]): int(offs[i] + lens[i])], i)
        g.flush()
        ds = g.device_stats()
    got = [res[i] for i in range(nm)]
    return {"devices": [device, device], "per_device_files": [d["files"] for d in ds],
            "parity": G.check_files("zipf10k", got, idx[:nm], hashed=True)}


def ingest_multi_leg(device: int = 0, max_file: int = 4 * M, nfiles: int = 1500) -> dict:
    """smoke()-sized check of the multi-device ingest front end
    (syncr_ingest_open_multi, devices {d, d}): the zipf10k files among the first
    `nfiles` that are at most `max_file` bytes, generated on the host (the
    corpus's xorshift rule), submitted from host memory, chunked + hashed, each
    compared with the golden digests."""
    import syncr_amd
    from oracle import oracle as O
    sizes = WL.zipf_sizes()
    rows = np.array([i for i in range(min(nfiles, sizes.size)) if int(sizes[i]) <= max_file], np.int64)
    host, offs = O.corpus_fill_threads(sizes[rows], indices=rows.astype(np.uint64))
    lens = sizes[rows]
    res: dict = {}
    with syncr_amd.Ingest(devices=[device, device], batch_bytes=16 << 20, depth=2, copy_threads=4,
                          on_file=lambda t, s, a: res.__setitem__(t, a)) as g:
        for j in range(rows.size):
            g.submit(host[int(offs[j]): int(offs[j] + lens[j])], j)
        g.flush()
        ds = g.device_stats()
    got = [res[j] for j in range(rows.size)]
    return {"devices": [device, device], "per_device_files": [d["files"] for d in ds],
            "parity": G.check_files("zipf10k", got, rows, hashed=True)}
