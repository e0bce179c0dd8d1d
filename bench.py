#!/usr/bin/env python3
"""bench.py -- device-resident Bup CDC throughput on MI355X.

Metric (BASELINE.json): GiB/s of file bytes chunked (bytes -> cut offsets),
inputs already resident in HBM, bit-exact vs the reference chunker.

One step = one pass of the hot path (scan kernel + dense pass + per-file
resolve, cuts written to HBM) over this rank's whole batch.  Workload at N=1:
SURVEY.md §8d config 3 -- 10 000 Zipf(1.5) files (4 KiB..128 MiB, 9.73 GiB).
With N GPUs the corpus is N such file sets (N x 10 000 files, distinct seeds),
LPT-sharded per file across ranks: fixed work per GPU ("weak" scaling), no
data-path collective (files are independent).  torch.distributed
(gloo) is used only for the barrier and the max-over-ranks of the step time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload zipf10k|uniform1k]
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s chunked device-resident (bytes→cut offsets); bit-exact vs ref"
METRIC_HASHED = "GiB/s chunked+BLAKE3-hashed device-resident (bytes→ChunkInfo); bit-exact vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
M = 1 << 20


def zipf_sizes(n: int = 10000, seed: int = 20251212) -> np.ndarray:
    """size_i = min(4 KiB * Z_i, 128 MiB), Z = rng.zipf(1.5)."""
    z = np.random.default_rng(seed).zipf(1.5, n).astype(np.float64)
    return np.minimum(4096.0 * z, float(128 * M)).astype(np.uint64)


def workload(name: str, world: int):
    """Global file table (sizes, corpus indices) for `world` GPUs."""
    if name == "zipf10k":
        one = zipf_sizes()
        desc = ("SURVEY §8d config 3: 10 000 Zipf(1.5) files, 4 KiB-128 MiB, 9.73 GiB per GPU; "
                "N GPUs chunk N x 10 000 files (distinct seeds) LPT-sharded per file (config 4)")
    elif name == "big1":
        one = np.full(1, 128 * M, np.uint64)
        desc = "diagnostic: one 128 MiB file (the longest resolve walk of zipf10k)"
    elif name == "uniform1k":
        one = np.full(1024, M, np.uint64)
        desc = "SURVEY §8d config 2: 1024 x 1 MiB files per GPU, LPT-sharded per file"
    else:
        raise SystemExit(f"unknown workload {name}")
    sizes = np.tile(one, world)
    return sizes, np.arange(sizes.size, dtype=np.uint64), desc


def lpt_shard(sizes: np.ndarray, world: int) -> list[np.ndarray]:
    """Longest-processing-time-first assignment of files to ranks."""
    order = np.argsort(-sizes.astype(np.int64), kind="stable")
    heap = [(0, r) for r in range(world)]
    parts: list[list[int]] = [[] for _ in range(world)]
    for i in order.tolist():
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return [np.array(sorted(p), dtype=np.int64) for p in parts]


class Dist:
    """Control plane only (barrier, max, sum) -- no data-path collective."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def reduce(self, x: float, op: str) -> float:
        if not self.pg:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op={"max": self.pg.ReduceOp.MAX, "sum": self.pg.ReduceOp.SUM}[op])
        return float(t.item())

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def load_traffic(workload_name: str, span: int, run_bytes: int):
    """HBM bytes per scan launch from the committed rocprofv3 PMC summary of
    the same workload, span and scan geometry (profiles/*_pmc_traffic.json)."""
    import glob
    import re

    def version(path):            # r01_v11h_pmc_traffic.json -> (1, 11): latest round/version last
        m = re.search(r"r(\d+)(?:_v(\d+))?", os.path.basename(path))
        return (int(m.group(1)), int(m.group(2) or 0)) if m else (0, 0)

    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")), key=version):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if (d.get("workload") == workload_name and int(d.get("span", -1)) == span
                and d.get("run_bytes") == run_bytes):
            best = d
    return best


def cpu_baseline(chunker, dbuf, offs, lens, cuts, sample_gib: float, hashed: bool = False):
    """Oracle (oracle/bup_oracle.c, the literal compute_file_chunks restatement)
    timed on this host on a bounded sample of the same bytes.  Also checks the
    GPU cuts of the sampled files against it.  hashed: the oracle also BLAKE3s
    every chunk (oracle/blake3_oracle.c) and the GPU hashes are checked."""
    from oracle import oracle as O
    take, tot = [], 0
    for i in range(lens.size):
        if tot >= sample_gib * 2**30:
            break
        take.append(i)
        tot += int(lens[i])
    take = np.array(take, dtype=np.int64)
    lo = int(offs[take[0]]) if take.size else 0
    hi = int(offs[take[-1]] + lens[take[-1]]) if take.size else 0
    host = dbuf.download(hi - lo, offset=lo)
    s_offs = (offs[take] - np.uint64(lo)).astype(np.uint64)
    s_lens = lens[take]
    def chunk_offsets(ref):
        o, n = [], []
        for j in range(take.size):
            ends = ref[j].astype(np.uint64)
            starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)[:ends.size]
            o.append(starts + s_offs[j])
            n.append(ends - starts)
        return (np.concatenate(o) if o else np.zeros(0, np.uint64),
                np.concatenate(n) if n else np.zeros(0, np.uint64))

    def run(nthreads):
        r = O.chunk_batch(host, s_offs, s_lens, nthreads=nthreads)
        hs = None
        if hashed:
            co, cn = chunk_offsets(r)
            hs = O.blake3_batch(host, co, cn, nthreads=nthreads)
        return r, hs

    t = time.perf_counter()
    ref, ref_h = run(1)
    dt1 = time.perf_counter() - t
    nthr = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    run(nthr)
    dtn = time.perf_counter() - t
    mism = 0
    k = 0
    for j, i in enumerate(take.tolist()):
        c = cuts[i]
        e = (c["offset"].astype(np.uint64) + c["len"].astype(np.uint64)).tolist()
        bad = e != ref[j].tolist()
        if hashed and not bad:
            bad = not np.array_equal(c["hash"], ref_h[k:k + c.size])
        k += c.size
        mism += bad
    gib = tot / 2**30
    return {
        "value": round(gib / dt1, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"first {take.size} files of rank 0's batch ({gib:.2f} GiB), production semantics, "
                  f"oracle/bup_oracle.c literal compute_file_chunks loop (gcc -O3), "
                  + ("plus oracle/blake3_oracle.c per chunk (portable C, no SIMD)" if hashed else "chunking only"),
        "threads_value": round(gib / dtn, 4), "threads": nthr,
        "gpu_cuts_match_sample": mism == 0, "sample_files_mismatched": int(mism),
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="zipf10k", choices=["zipf10k", "uniform1k", "big1"])
    ap.add_argument("--mode", default="production", choices=["production", "ideal"])
    ap.add_argument("--cpu-sample-gib", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-read-probe", action="store_true",
                    help="skip the streaming-read microbenchmark reported as roofline.measured_read_peak")
    ap.add_argument("--pipeline-depth", type=int, default=2,
                    help="after the timed region, also time K steps with this many batches in flight "
                         "(each slot its own engine handle, HIP stream and copy of the corpus, like the "
                         "ingest pipeline's slots); reported as `pipelined`, 1 = skip")
    ap.add_argument("--hashed", action="store_true",
                    help="also BLAKE3 every chunk on the GPU (SURVEY §8f next #1); reports the "
                         "chunk+hash rate as its own metric, not the BASELINE metric")
    args = ap.parse_args(argv)

    d = Dist()
    world = d.world
    import syncr_amd
    read_cap = syncr_amd.TOKIO_READ_CAP if args.mode == "production" else 0
    ch = syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, read_cap, device=d.local_rank)

    sizes, indices, desc = workload(args.workload, world)
    mine = lpt_shard(sizes, world)[d.rank]
    lens = sizes[mine]
    idx = indices[mine]
    offs = np.zeros_like(lens)
    if lens.size:
        offs[1:] = np.cumsum(lens)[:-1]
    span = int(lens.sum())
    depth = max(1, args.pipeline_depth)
    slots = []                                # (handle, corpus copy): one batch in flight each
    for k in range(depth):
        h = ch if k == 0 else syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, read_cap,
                                                 device=d.local_rank)
        b = syncr_amd.DeviceBuffer(h, span)   # own buffer: no slot reads another's bytes from cache
        b.gen_corpus(offs, lens, indices=idx)
        h.plan(offs, lens, span)
        slots.append((h, b))
    ch, dbuf = slots[0]

    def run_steps(nslots, steps):
        for k in range(steps):
            h, b = slots[k % nslots]
            h.launch(b.ptr, hashed=args.hashed)
        for h, _ in slots[:nslots]:
            h.synchronize()

    run_steps(1, args.warmup)
    d.barrier()
    ch.synchronize()
    ch.set_timing(True, scan_only=True)       # HIP events around the scan kernel, on its stream
    t0 = time.perf_counter()
    run_steps(1, args.steps)                  # the timed region: one batch in flight
    dt = time.perf_counter() - t0
    d.barrier()
    kms, nl = ch.kernel_times()
    ch.set_timing(False)
    # diagnostics outside the timed region: every phase bracketed by events
    ch.set_timing(True)
    run_steps(1, min(args.steps, 5))
    pms, pn = ch.kernel_times()
    ch.set_timing(False)

    pipelined = None
    if depth > 1:                             # the same K steps with `depth` batches in flight
        run_steps(depth, max(args.warmup, depth))
        d.barrier()
        t0 = time.perf_counter()
        run_steps(depth, args.steps)
        dtp = d.reduce(time.perf_counter() - t0, "max")
        d.barrier()
        stepp = dtp / max(args.steps, 1)
        pipelined = {"depth": depth, "value": round(d.reduce(float(span), "sum") / stepp / 2**30, 3),
                     "ms_per_step": round(stepp * 1e3, 4),
                     "note": "same workload and K; step k on slot k % depth, each slot its own handle, "
                             "HIP stream and corpus copy; per-launch kernel times overlap here, so the "
                             "roofline is taken from the one-in-flight timed region"}

    dt_max = d.reduce(dt, "max")
    total_bytes = d.reduce(float(span), "sum")
    step_s = dt_max / max(args.steps, 1)
    value = total_bytes / step_s / 2**30

    cuts = ch.fetch(hashed=args.hashed)
    slots_agree = all(all(np.array_equal(a, x) for a, x in zip(cuts, h.fetch(hashed=args.hashed)))
                      for h, _ in slots[1:])
    stats = ch.last_stats()
    engine_info = ch.info()
    ncuts = int(sum(c.size for c in cuts))
    covered = all(int(c["len"].sum()) == int(n) for c, n in zip(cuts, lens.tolist()))

    scan_ms = kms[0] / max(nl, 1)
    achieved = span / (scan_ms / 1e3) / 1e9 if scan_ms > 0 else 0.0
    tr = load_traffic(args.workload, span, engine_info["run_bytes"])
    roofline = {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": (int(tr["hbm_bytes_per_launch"]) if tr else None),
        "kernel": engine_info["scan_kernel"], "kernel_ms": round(scan_ms, 4),
        "algorithmic_bytes_per_launch": span,
        "dense_ms": round(pms[1] / max(pn, 1), 4), "resolve_ms": round(pms[2] / max(pn, 1), 4),
        "hash_ms": round(pms[3] / max(pn, 1), 4) if args.hashed else None,
        "traffic_source": (tr.get("source") if tr else None),
    }
    if not args.no_read_probe and span >= 16:
        # measured streaming-read ceiling over the same resident bytes:
        # a read-only kernel, best pass of `reps`, both load policies
        probe = {}
        for nt in (True, False):
            best, mean = ch.read_probe(dbuf.ptr, span, reps=10, nt=nt)
            probe["nt" if nt else "plain"] = {"best_gbs": round(span / (best / 1e3) / 1e9, 1),
                                              "mean_gbs": round(span / (mean / 1e3) / 1e9, 1)}
        peak_meas = max(v["best_gbs"] for v in probe.values())
        roofline["measured_read_peak"] = peak_meas
        roofline["frac_of_measured"] = round(achieved / peak_meas, 4) if peak_meas else None
        roofline["read_probe"] = dict(probe, kernel="cdc_read_probe_kernel (syncr_cdc_read_probe), 10 passes "
                                                    "over the corpus buffer, 16 B loads, no writes")
    cpu = None
    if d.rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ch, dbuf, offs, lens, cuts, args.cpu_sample_gib, hashed=args.hashed)
    for h, b in slots:
        b.free()
        h.close()

    if d.rank == 0:
        out = {
            "metric": METRIC_HASHED if args.hashed else METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: per-file xorshift64 corpus generated in HBM (SURVEY §8d seed rule)",
            "config": {
                "workload": f"{args.workload}: {desc}", "files_per_gpu": int(lens.size),
                "bytes_per_gpu": span, "total_bytes": int(total_bytes), "chunk_bits": 20,
                "max_chunk": syncr_amd.MAX_CHUNK_SIZE, "read_cap": read_cap, "mode": args.mode,
                "parallelism": f"file-sharded x{world} (LPT), one HIP stream per GPU, no collective",
                "slots_agree_rank0": slots_agree,
                "cuts_rank0": ncuts, "coverage_ok_rank0": covered,
                "candidates_rank0": int(stats["candidates"]), "dense_tiles_rank0": int(stats["dense_tiles"]),
                "engine": engine_info,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pipelined": pipelined,
        }
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()
