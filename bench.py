#!/usr/bin/env python3
"""bench.py -- device-resident Bup CDC throughput on MI355X.

Metric (BASELINE.json): GiB/s of file bytes chunked (bytes -> cut offsets),
inputs already resident in HBM, bit-exact vs the reference chunker.

One step = one pass of the hot path (scan kernel + dense pass + compaction +
per-file resolve, cuts written to HBM) over this rank's whole batch.  Workload
at N=1: SURVEY.md §8d config 3 -- 10 000 Zipf(1.5) files (4 KiB..128 MiB,
9.73 GiB).  With N GPUs (BASELINE config 4) the SAME 10 000-file corpus is
LPT-sharded per file across the ranks (`--scaling strong`, the default): the
aggregate is the corpus bytes / the max per-rank step time.  `--scaling weak`
gives every rank its own 10 000 files instead.  No data-path collective: files
are independent; torch.distributed (gloo) carries only the
barrier and the max / sum / gather of per-rank numbers.

After the timed headline (untimed, N=1 only, on the same GPU): the parity leg
-- every file of the headline corpus in both semantics and with hashes against
golden digests, every KAT case, the BLAKE3 vectors, an adversarial subset, the
multi-device ingest -- and the other single-GPU BASELINE configs: uniform1k
(config 2), dedup (config 5), the adversarial dense workload, and the
end-to-end ingest rate from host memory.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]
                    [--workload zipf10k|uniform1k|dense|big1|dense1|dedup]

`--gpus N` with N > 1 launches the N ranks itself (one process per GPU, before
anything touches HIP) unless a launcher (torchrun) already set WORLD_SIZE, in
which case WORLD_SIZE must equal N.  `--dry-run` does everything but touch a
device: it prints the shard plan (files / bytes per rank, disjointness).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from benchlib.workloads import (DENSE_CONSTANT, DENSE_PERIODIC, WORKLOADS, dedup_plan, dense_kind,  # noqa: E402,F401
                                lpt_shard, offsets_of, periodic_pattern, workload, zipf_sizes)

METRIC = "GiB/s chunked device-resident (bytes→cut offsets); bit-exact vs ref"
METRIC_HASHED = "GiB/s chunked+BLAKE3-hashed device-resident (bytes→ChunkInfo); bit-exact vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
M = 1 << 20
# golden digest fixture of each workload's corpus (tests/golden/<name>_digests.npz)
GOLDEN_OF = {"zipf10k": "zipf10k", "dense": "dense", "dedup": "dedup"}


class Dist:
    """Control plane only (barrier, max, sum, gather) -- no data-path collective."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # Gloo reports its connections on stdout ("[Gloo] Rank r is connected
            # to ..."), which would mix into the one JSON line rank 0 prints:
            # send fd 1 to stderr while the group connects
            import ctypes
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            finally:
                ctypes.CDLL(None).fflush(None)
                os.dup2(saved, 1)
                os.close(saved)
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

    def gather(self, obj) -> list:
        if not self.pg:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """One process per GPU, started here before anything touches HIP (the
    parent never initialises a device).  Each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* like torchrun would set them; rank 0 prints the line.
    A failing rank stops the others (by their exact PIDs)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def load_traffic(workload_name: str, span: int, run_bytes: int, kernel: str = "cdc::cdc_scan_kernel",
                 st_segments: int | None = None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    of the same workload, span and scan geometry (profiles/*_pmc_traffic.json);
    for the stream-tile scan also the same segments per stream (summaries
    without the key were measured with 9)."""
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
        dk = d.get("kernel", "cdc::cdc_scan_kernel")     # the summary's main kernel
        if (d.get("workload") == workload_name and int(d.get("span", -1)) == span
                and d.get("run_bytes") == run_bytes
                and (kernel == dk or kernel in d.get("per_kernel_hbm_bytes", {}))
                and (not st_segments or kernel != dk or int(d.get("st_segments") or 9) == st_segments)):
            best = dict(d)
            best["hbm_bytes_per_launch"] = (d["hbm_bytes_per_launch"] if kernel == dk
                                            else d["per_kernel_hbm_bytes"][kernel])
    return best


def cpu_host() -> dict:
    """The host the CPU baseline runs on (state core count and model)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    share = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_share": share,
            "cpu_share_source": "OMP_NUM_THREADS (the GPU box's CPU share per GPU)" if omp else "sched_getaffinity"}


def cpu_baseline(dbuf, offs, lens, cuts, hcuts, sample_gib: float, skip=None):
    """Oracle (oracle/bup_oracle.c, the literal compute_file_chunks restatement)
    timed on this host on a bounded sample of the same bytes, single thread (the
    reference's serial per-file loop) and on every core of this job's CPU share.
    Also the checker of the sample: the GPU cuts (and, when hcuts is given, the
    GPU BLAKE3 of every chunk: oracle/blake3_oracle.c) must match it bit for bit.
    skip(i): files left out of the sample (see the `sample` text)."""
    from oracle import oracle as O
    take, tot, skipped = [], 0, 0
    for i in range(lens.size):
        if tot >= sample_gib * 2**30:
            break
        if skip is not None and skip(i):
            skipped += 1
            continue
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

    hw = cpu_host()
    nthr = hw["cpu_share"]
    t = time.perf_counter()
    ref = O.chunk_batch(host, s_offs, s_lens, nthreads=1)
    dt1 = time.perf_counter() - t
    t = time.perf_counter()
    O.chunk_batch(host, s_offs, s_lens, nthreads=nthr)
    dtn = time.perf_counter() - t
    # SURVEY §8d's "one file per thread on all nproc cores" leg: every CPU this
    # process may run on (sched_getaffinity), a burst of well under a second
    nall = max(1, min(int(hw["affinity_cpus"] or 1), 512))
    t = time.perf_counter()
    O.chunk_batch(host, s_offs, s_lens, nthreads=nall)
    dta = time.perf_counter() - t
    mism = 0
    for j, i in enumerate(take.tolist()):
        c = cuts[i]
        e = (c["offset"].astype(np.uint64) + c["len"].astype(np.uint64)).tolist()
        mism += e != ref[j].tolist()
    gib = tot / 2**30
    nproc = hw["nproc"] or nthr
    out = {
        "value": round(gib / dt1, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"first {take.size} files of rank 0's batch ({gib:.2f} GiB), production semantics, "
                  f"oracle/bup_oracle.c literal compute_file_chunks loop (gcc -O3), chunking only; "
                  f"`value` single thread (the reference chunks one file at a time, file_operations.rs:599-605), "
                  f"`threads_value` one file per thread on `threads` threads",
        "threads_value": round(gib / dtn, 4), "threads": nthr, **hw,
        # (the key says what bounds it: one file per thread, so the sample's largest file -- chunked
        # serially, as the reference does -- sets the time however many cores there are)
        "all_cores_value_bounded_by_largest_file": round(gib / dta, 4), "all_cores_threads": nall,
        "all_cores_largest_file_bytes": int(s_lens.max()) if s_lens.size else 0,
        "all_cores_note": (f"SURVEY §8d's 'one file per thread on all nproc cores' leg, measured: {nall} threads "
                           f"(every CPU in this process's affinity mask; nproc {nproc}) over the same sample; "
                           f"the largest sample file's serial walk bounds it (one file per thread, as the "
                           f"reference chunks a file serially), so it can read below threads_value"),
        "gpu_cuts_match_sample": mism == 0, "sample_files_mismatched": int(mism),
    }
    if skip is not None:
        out["sample_files_skipped"] = skipped
    if hcuts is not None:
        co, cn = chunk_offsets(ref)
        t = time.perf_counter()
        ref_h = O.blake3_batch(host, co, cn, nthreads=nthr)
        dth = time.perf_counter() - t
        hm, k = 0, 0
        for i in take.tolist():
            c = hcuts[i]
            hm += not np.array_equal(c["hash"], ref_h[k:k + c.size])
            k += c.size
        out["hashed_threads_value"] = round(gib / (dtn + dth), 4)
        out["gpu_hashes_match_sample"] = hm == 0 and k == ref_h.shape[0]
        out["sample_chunks_hashed"] = int(k)
    return out


def dry_run(d: Dist, args) -> None:
    sizes, idx, desc = workload(args.workload, d.world, args.scaling)
    mine = lpt_shard(sizes, d.world)[d.rank]
    plan = d.gather({"rank": d.rank, "files": mine.tolist()})
    if d.rank == 0:
        allf = np.concatenate([np.array(p["files"], np.int64) for p in plan]) if plan else np.zeros(0, np.int64)
        loads = [int(sizes[np.array(p["files"], np.int64)].sum()) for p in plan]
        print(json.dumps({
            "dry_run": True, "n_gpus": d.world, "workload": args.workload, "scaling": args.scaling,
            "total_files": int(sizes.size), "total_bytes": int(sizes.sum()),
            "shards": [{"rank": p["rank"], "files": len(p["files"]), "bytes": l} for p, l in zip(plan, loads)],
            "disjoint": bool(np.unique(allf).size == allf.size),
            "covers_all": bool(np.array_equal(np.sort(allf), np.arange(sizes.size))),
            "max_over_mean": round(max(loads) / (sum(loads) / len(loads)), 5) if loads and sum(loads) else None,
            "launcher": os.environ.get("SYNCR_BENCH_LAUNCHER", "env"),
        }), flush=True)


def run_legs(args, dev_id: int, dbuf, offs, lens, idx, rank_span: int, out: dict) -> None:
    """N=1 only, after the headline: parity legs and the other single-GPU configs."""
    from benchlib import legs as L
    t_all = time.perf_counter()
    parity = out.setdefault("parity", {})
    timing = {}

    def timed(name, fn, *a):
        t = time.perf_counter()
        try:
            r = fn(*a)
        except Exception as e:                                   # reported, never hidden
            r = {"error": f"{type(e).__name__}: {e}"}
        timing[name] = round(time.perf_counter() - t, 2)
        return r

    if args.workload == "zipf10k":
        parity["ideal"] = timed("ideal", L.ideal_leg, dbuf, offs, lens, idx, dev_id)
        host = dbuf.download(rank_span)
    else:
        host = None
    for h, b in out.pop("_slots"):
        b.free()
        h.close()
    parity["kat"] = timed("kat", L.kat_leg, dev_id)
    parity["blake3_vectors"] = timed("blake3_vectors", L.blake3_vectors_leg, dev_id)
    parity["dense_subset"] = timed("dense_subset", L.dense_subset_leg, dev_id)
    k, w = args.steps, max(args.warmup, 2)
    if args.workload == "zipf10k":
        # BASELINE config 4's per-rank batch (zipf10k / 8, LPT) timed on this GPU
        out["shard8"] = timed("shard8", L.shard_leg, dev_id, k, w, 8)
    if args.workload != "uniform1k":
        out["uniform1k"] = timed("uniform1k", L.uniform1k_leg, dev_id, k, w)
    if args.workload != "dedup":
        out["dedup"] = timed("dedup", L.dedup_leg, dev_id, k, w)
    if args.workload != "dense":
        out["dense"] = timed("dense", L.dense_leg, dev_id, k, w)
    if args.workload != "dense1":
        out["dense1"] = timed("dense1", L.dense1_leg, dev_id, k, w)
    out["h2d_probe"] = timed("h2d_probe", L.h2d_probe, dev_id)
    if host is not None:
        # end to end from host memory / files, driven from C++ (benchlib/e2e_driver.cpp): the
        # shim's per-file call site, the batched walk, and the ingest entry points
        from benchlib import e2e as E
        e2e = timed("e2e", E.legs, host, offs, lens, idx, dev_id)
        for key in E.MODES:
            out[key] = e2e.get(key, {"error": e2e.get("error", "not run")})
        md = timed("ingest_multi_device", L.ingest_multi_device_leg, host, offs, lens, idx, dev_id)
        parity["ingest_multi_device"] = md.get("parity", md)
        h2d = out["h2d_probe"].get("h2d", {}).get("best_gbs")
        cpu1 = (out.get("cpu_baseline") or {}).get("value")
        for key in E.MODES:
            v = out[key].get("value")
            if h2d and v:          # the end-to-end rate on its link ceiling (GiB/s -> GB/s)
                out[key]["frac_of_h2d"] = round(v * 2**30 / 1e9 / h2d, 4)
            if cpu1 and v:         # next to the reference loop's one-thread rate (cpu_baseline.value)
                out[key]["vs_cpu_one_thread"] = round(v / cpu1, 2)
    del host
    # one summary: every parity check of the line
    checks = []
    for name, p in list(parity.items()) + [(f"{s}.parity", out.get(s, {}).get("parity")) for s in
                                            ("shard8", "uniform1k", "dedup", "dense", "dense1", "ingest",
                                             "ingest_files", "ingest_zero_copy", "shim_per_file", "shim_walk")] + \
            [(f"{s}.parity_hashed", out.get(s, {}).get("parity_hashed")) for s in ("dedup", "dense", "dense1")] + \
            [("dense1.parity_ideal", out.get("dense1", {}).get("parity_ideal"))]:
        if isinstance(p, dict) and "mismatches" in p:
            checks.append((name, p.get("files", p.get("cases", 0)), p["mismatches"] + p.get("hash_mismatches", 0)))
        elif isinstance(p, dict):
            checks.append((name, 0, 1))                          # error / missing fixture: counted as a failure
    parity["summary"] = {"checks": len(checks), "files_or_cases": int(sum(c[1] for c in checks)),
                         "mismatches": int(sum(c[2] for c in checks)),
                         "failed": [c[0] for c in checks if c[2]]}
    out["legs_seconds"] = dict(timing, total=round(time.perf_counter() - t_all, 2))


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="zipf10k", choices=list(WORKLOADS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="N>1: strong = one file set sharded across the ranks (BASELINE config 4, default); "
                         "weak = one file set per rank")
    ap.add_argument("--mode", default="production", choices=["production", "ideal"])
    ap.add_argument("--cpu-sample-gib", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the untimed parity leg and the other BASELINE configs (N=1)")
    ap.add_argument("--no-read-probe", action="store_true",
                    help="skip the streaming-read microbenchmark reported as roofline.measured_read_peak")
    ap.add_argument("--pipeline-depth", type=int, default=2,
                    help="after the timed region, also time K steps with this many batches in flight "
                         "(each slot its own engine handle, HIP stream and copy of the corpus, like the "
                         "ingest pipeline's slots); reported as `pipelined`, 1 = skip")
    ap.add_argument("--hashed", action="store_true",
                    help="make the chunk+BLAKE3 rate the headline (profiling the hash kernels); by default "
                         "it is reported in the `hashed` sub-object after the headline region")
    ap.add_argument("--no-hashed", action="store_true", help="skip the `hashed` sub-object")
    ap.add_argument("--sustained-steps", type=int, default=80,
                    help="untimed steps before the `sustained` re-timing of K steps (0 = skip)")
    ap.add_argument("--dry-run", action="store_true", help="shard plan only, no device")
    ap.add_argument("--device-map", default=None,
                    help="rehearsal only: comma-separated device per local rank (e.g. 0,0 runs two ranks on one "
                         "GPU); default: device = LOCAL_RANK")
    ap.add_argument("--fetch-at", default="after", choices=["first", "end", "after"],
                    help="where the results are first fetched (capacity re-runs settle there): after the timed "
                         "region (default: no host gap anywhere between the first warm-up step and the timed "
                         "steps; re-timed if that fetch had to re-run), after warm-up step 1, or after the last")
    ap.add_argument("--dev-lib", action="store_true",
                    help="tools/ only: run against libsyncr_cdc_dev.so (variants / ablations by env)")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        os.environ["SYNCR_BENCH_LAUNCHER"] = "bench.py"
        return spawn_ranks(args.gpus, argv)
    d = Dist()
    world = d.world
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dry_run(d, args)
        d.close()
        return 0

    import syncr_amd
    from benchlib import golden as G
    from benchlib import legs as L
    if args.dev_lib:
        syncr_amd.use_dev_library()
    read_cap = syncr_amd.TOKIO_READ_CAP if args.mode == "production" else 0
    dev_id = d.local_rank
    if args.device_map:
        dmap = [int(x) for x in args.device_map.split(",")]
        if len(dmap) < world:
            raise SystemExit(f"--device-map names {len(dmap)} devices for {world} ranks")
        dev_id = dmap[d.local_rank]
    ch = syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, read_cap, device=dev_id)

    sizes, indices, desc = workload(args.workload, world, args.scaling)
    mine = lpt_shard(sizes, world)[d.rank]
    lens = sizes[mine]
    idx = indices[mine]
    offs = offsets_of(lens)
    span = int(lens.sum())
    depth = max(1, args.pipeline_depth)

    def make_slot(h):
        """A handle with its own copy of the corpus (one batch in flight each)."""
        b = syncr_amd.DeviceBuffer(h, max(span, 16))   # own buffer: no slot reads another's bytes from cache
        if args.workload == "dedup":
            plan = dedup_plan()
            L.build_dedup(h, b, offs, [plan[int(i) % len(plan)] for i in idx.tolist()])
        else:
            b.gen_corpus(offs, lens, indices=idx)
        if args.workload == "dense":
            L.fill_dense(b, offs, lens, idx)
        elif args.workload == "dense1":
            b.upload(np.resize(periodic_pattern(), span))
        h.plan(offs, lens, span)
        return (h, b)

    # the headline runs with ONE handle open on the device (one batch in
    # flight, like a single chunking thread); the pipelined section below adds
    # the other slots' handles
    slots = [make_slot(ch)]
    ch, dbuf = slots[0]
    head_hashed = args.hashed

    def run_steps(nslots, steps, hashed=head_hashed):
        for k in range(steps):
            h, b = slots[k % nslots]
            h.launch(b.ptr, hashed=hashed)
        for h, _ in slots[:nslots]:
            h.synchronize()

    # W warm-up steps in all; results are fetched once inside them so a
    # capacity re-run settles before timing.  Fetching after the FIRST warm-up
    # step keeps the host-side gap (D2H + host work) away from the timed
    # region: on MI355X the shader clock dips for ~20 launches whenever the
    # scan load resumes after a gap (profiles/r02_v2_dispatches.json)
    def warm_and_time(fetch_at):
        if fetch_at == "first" and args.warmup > 0:
            run_steps(1, 1)
            ch.fetch(hashed=head_hashed)
            run_steps(1, args.warmup - 1)
        elif fetch_at == "after":
            run_steps(1, args.warmup)
        else:
            run_steps(1, args.warmup)
            ch.fetch(hashed=head_hashed)
        d.barrier()
        ch.synchronize()
        # the scan kernel timed by the device clock inside the kernel (no event packets in the
        # queue: the timed steps run exactly as untimed ones); HIP events cross-check below
        ch.set_timing(True, scan_only=True)
        t0 = time.perf_counter()
        run_steps(1, args.steps)                  # the timed region: one batch in flight
        dt = time.perf_counter() - t0
        d.barrier()
        kms, nl = ch.kernel_times()
        ch.set_timing(False)
        return dt, kms, nl, ch.last_scan()      # the library's own report of the scan it ran

    # The host-side fetch (D2H + list building) is a gap of the device's load,
    # and on MI355X the shader clock dips whenever the scan load resumes after a
    # gap (§4.2): by default nothing is fetched between the first warm-up step
    # and the timed steps (profiles/r03_ab_fetch_gap.log: +0.8-1.3 %).  The
    # first fetch comes after the timed region; if it had to re-run a launch
    # with grown capacities, the timed launches ran with the smaller ones, so the
    # region is timed again (now with settled capacities, fetch after step 1).
    fetch_mode = args.fetch_at
    dt, kms, nl, scan_info = warm_and_time(fetch_mode)
    retimed = False
    if fetch_mode == "after":
        ch.fetch(hashed=head_hashed)
        if d.reduce(float(ch.fetch_reruns()), "max") > 0:
            fetch_mode, retimed = "first", True
            dt, kms, nl, scan_info = warm_and_time(fetch_mode)
    # diagnostics outside the timed region: every phase bracketed by events
    ch.set_timing(True)
    run_steps(1, min(args.steps, 5))
    pms, pn = ch.kernel_times()
    ch.set_timing(False)
    # cross-check of the device-clock scan time: the same K steps with HIP events bound to the
    # scan's dispatch on its launch stream (each event pair adds queue idle to a step)
    ch.set_timing(True, scan_only=True, events=True)
    run_steps(1, args.steps)
    ems, en = ch.kernel_times()
    ch.set_timing(False)

    dt_max = d.reduce(dt, "max")
    total_bytes = d.reduce(float(span), "sum")
    step_s = dt_max / max(args.steps, 1)
    value = total_bytes / step_s / 2**30

    # sustained rate: the same one-in-flight steps after ~150 ms of back-to-back
    # chunking.  On MI355X the shader clock dips for the first ~30 ms of a
    # sustained scan (2.1 -> 1.7 GHz by rocprofv3 GRBM_GUI_ACTIVE)
    # and the timed K steps above usually start inside that dip; a continuously
    # running ingest pipeline sees this rate.
    sustained = None
    if args.sustained_steps:
        run_steps(1, args.sustained_steps)
        d.barrier()
        ch.synchronize()
        ch.set_timing(True, scan_only=True)
        t0 = time.perf_counter()
        run_steps(1, args.steps)
        dts = d.reduce(time.perf_counter() - t0, "max")
        d.barrier()
        sms, sn = ch.kernel_times()
        ch.set_timing(False)
        steps_s = dts / max(args.steps, 1)
        sustained = {"value": round(total_bytes / steps_s / 2**30, 3), "ms_per_step": round(steps_s * 1e3, 4),
                     "scan_ms": round(sms[0] / max(sn, 1), 4),
                     "scan_frac": round(span / (sms[0] / max(sn, 1) / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if sn else None,
                     "note": f"the same K one-in-flight steps, timed after {args.sustained_steps} more untimed steps "
                             "(past the shader-clock dip of the first ~30 ms of sustained scanning); not the "
                             "headline `value`"}

    pipelined = None
    if depth > 1:                             # the same K steps with `depth` batches in flight
        for _ in range(depth - 1):
            slots.append(make_slot(syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, read_cap,
                                                     device=dev_id)))
        for h, b in slots[1:]:                # settle capacity re-runs before timing
            h.launch(b.ptr, hashed=head_hashed)
            h.fetch(hashed=head_hashed)
        run_steps(depth, max(args.warmup, depth))
        d.barrier()
        t0 = time.perf_counter()
        run_steps(depth, args.steps)
        dtp = d.reduce(time.perf_counter() - t0, "max")
        d.barrier()
        stepp = dtp / max(args.steps, 1)
        pipelined = {"depth": depth, "value": round(total_bytes / stepp / 2**30, 3),
                     "ms_per_step": round(stepp * 1e3, 4),
                     "note": "same workload and K; step k on slot k % depth, each slot its own handle, "
                             "HIP stream and corpus copy; a slot's scan waits for the previous slot's scan "
                             "(scans fill the GPU), the compaction/resolve tails overlap the next scan; "
                             "the roofline is taken from the one-in-flight timed region"}

    cuts = ch.fetch(hashed=head_hashed)
    slots_agree = all(all(np.array_equal(a, x) for a, x in zip(cuts, h.fetch(hashed=head_hashed)))
                      for h, _ in slots[1:])
    stats = ch.last_stats()
    engine_info = ch.info()
    ncuts = int(sum(c.size for c in cuts))
    covered = all(int(c["len"].sum()) == int(n) for c, n in zip(cuts, lens.tolist()))

    scan_ms = kms[0] / max(nl, 1)
    achieved = span / (scan_ms / 1e3) / 1e9 if scan_ms > 0 else 0.0
    scan_kernel = scan_info["kernel"]           # syncr_cdc_last_scan of the last timed launch
    tr = load_traffic(args.workload, span, engine_info["run_bytes"], kernel="cdc::" + scan_kernel,
                      st_segments=scan_info.get("st_segments"))
    roofline = {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": (int(tr["hbm_bytes_per_launch"]) if tr else None),
        "kernel": scan_kernel, "kernel_ms": round(scan_ms, 4), "scan_schedule": scan_info,
        "kernel_timing": "mean over the K timed launches by the device clock (the scan's waves stamp "
                         "wall_clock64 at entry / exit, syncr_cdc_set_timing mode 4: no queue packets); "
                         "kernel_ms_hip_events: the same K steps right after, HIP events bound to the scan "
                         "dispatch on its stream",
        "kernel_ms_hip_events": round(ems[0] / max(en, 1), 4) if en else None,
        "algorithmic_bytes_per_launch": span,
        "dense_ms": round(pms[1] / max(pn, 1), 4), "resolve_ms": round(pms[2] / max(pn, 1), 4),
        "hash_ms": round(pms[3] / max(pn, 1), 4) if head_hashed else None,
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

    # complete ChunkInfo records (boundaries + BLAKE3 of every chunk, the
    # hash_binary call at file_operations.rs:757): timed after the headline
    # region, on the same corpus, one batch in flight
    hashed = None
    hcuts = None
    if not args.no_hashed and not head_hashed:
        run_steps(1, max(1, min(args.warmup, 3)), hashed=True)
        ch.fetch(hashed=True)
        d.barrier()
        ch.synchronize()
        t0 = time.perf_counter()
        run_steps(1, args.steps, hashed=True)
        dth = d.reduce(time.perf_counter() - t0, "max")
        d.barrier()
        ch.set_timing(True)
        run_steps(1, min(args.steps, 5), hashed=True)
        hms, hn = ch.kernel_times()
        ch.set_timing(False)
        hcuts = ch.fetch(hashed=True)
        steph = dth / max(args.steps, 1)
        hpipe = None
        if depth > 1:                             # the same K hashed steps, `depth` batches in flight
            for h, b in slots[1:]:
                h.launch(b.ptr, hashed=True)
                h.fetch(hashed=True)
            run_steps(depth, max(args.warmup, depth), hashed=True)
            d.barrier()
            t0 = time.perf_counter()
            run_steps(depth, args.steps, hashed=True)
            dthp = d.reduce(time.perf_counter() - t0, "max")
            d.barrier()
            hpipe = round(total_bytes / (dthp / max(args.steps, 1)) / 2**30, 3)
        hash_ms = hms[3] / max(hn, 1)
        htr = load_traffic(args.workload, span, engine_info["run_bytes"], kernel="cdc::b3_leaf_kernel")
        hashed = {
            "metric": METRIC_HASHED, "value": round(total_bytes / steph / 2**30, 3), "unit": "GiB/s",
            "ms_per_step": round(steph * 1e3, 4), "hash_ms": round(hash_ms, 4),
            "scan_ms": round(hms[0] / max(hn, 1), 4),
            "hash_rate_gbs": round(span / (hash_ms / 1e3) / 1e9, 1) if hash_ms > 0 else None,
            "cuts_agree_with_headline": all(np.array_equal(a[f], x[f]) for a, x in zip(hcuts, cuts)
                                            for f in ("offset", "len", "file")),
            "pipelined_value": hpipe,
            "leaf_traffic_over_algorithmic": (round(htr["hbm_bytes_per_launch"] / span, 4) if htr else None),
            "leaf_traffic_source": (htr.get("source") if htr else None),
            "sample_check": "cpu_baseline.gpu_hashes_match_sample (rank 0, N=1) and parity.headline_hashed",
        }

    # parity of the headline corpus: every file of this rank against the golden
    # digests of the CPU oracle (weak-scaled copies with other seeds are skipped)
    parity = {}
    gname = GOLDEN_OF.get(args.workload)
    if gname is not None:
        rows = idx.astype(np.int64) % (1000 if gname == "dedup" else 1 << 62)
        sem = "production" if read_cap else "ideal"
        parity["headline"] = G.check_files(gname, cuts, rows, semantics=sem, hashed=head_hashed)
        if hcuts is not None:
            parity["headline_hashed"] = G.check_files(gname, hcuts, rows, semantics=sem, hashed=True)
    ranks = d.gather({"rank": d.rank, "device": dev_id, "files": int(lens.size), "bytes": span,
                      "ms_per_step": round(dt / max(args.steps, 1) * 1e3, 4), "scan_ms": round(scan_ms, 4),
                      "scan_frac": round(achieved / HBM_PEAK_GBS, 4), "parity": parity})
    if world > 1:
        for key in ("headline", "headline_hashed"):
            ps = [r["parity"].get(key) for r in ranks if r["parity"].get(key)]
            if ps:
                parity[key] = {"files": sum(p.get("files", 0) for p in ps),
                               "chunks": sum(p.get("chunks", 0) for p in ps),
                               "mismatches": sum(p.get("mismatches", 0) for p in ps),
                               "fixture": ps[0].get("fixture"), "ranks": len(ps)}

    cpu = None
    # dense1 is one periodic file: the literal loop would memmove 16 MiB per 64-byte chunk
    if d.rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload != "dense1":
        skip = None
        if args.workload == "dense":
            # the literal loop memmoves its buffer (copy_within, file_operations.rs:771)
            # after every 64-byte chunk of a periodic file: quadratic in the file
            # size, hours for the 128 MiB ones; the sample keeps those up to 1 MiB
            skip = lambda i: dense_kind(int(idx[i])) == 1 and int(lens[i]) > (1 << 20)   # noqa: E731
        cpu = cpu_baseline(dbuf, offs, lens, cuts, hcuts, args.cpu_sample_gib, skip=skip)
        if skip is not None:
            cpu["sample"] += "; periodic files over 1 MiB skipped (the literal loop's memmove per 64-byte chunk)"

    out = {
        "metric": METRIC_HASHED if head_hashed else METRIC, "value": round(value, 3), "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u8",
        "data": ("synthetic: one random 32 MiB base (corpus file DEDUP_BASE_INDEX, generated in HBM) and its "
                 "single-edit variants, copied together in HBM" if args.workload == "dedup" else
                 "synthetic: per-file xorshift64 corpus generated in HBM (SURVEY §8d seed rule)"
                 + ("; adversarial files uploaded from the host (dense_kind)" if args.workload == "dense" else "")),
        "config": {
            "workload": f"{args.workload}: {desc}", "files_per_gpu": int(lens.size),
            "bytes_per_gpu": span, "total_files": int(sizes.size), "total_bytes": int(total_bytes),
            "chunk_bits": 20, "max_chunk": syncr_amd.MAX_CHUNK_SIZE, "read_cap": read_cap, "mode": args.mode,
            "parallelism": (f"file-sharded x{world} (LPT, {args.scaling} scaling), one process + HIP stream per "
                            "GPU, no collective"),
            "launcher": os.environ.get("SYNCR_BENCH_LAUNCHER", "torchrun/env" if world > 1 else "none"),
            "device_map": args.device_map or "device = LOCAL_RANK",
            "warmup_fetch": ("results first fetched after the timed region (no host gap from warm-up step 1 "
                             "through the timed steps); no capacity re-run was needed" if fetch_mode == "after" else
                             f"results fetched after warm-up step {1 if fetch_mode == 'first' else args.warmup} of "
                             f"{args.warmup}" + ("; re-timed: the first fetch had to re-run with grown capacities"
                                                  if retimed else "")),
            "slots_agree_rank0": slots_agree,
            "cuts_rank0": ncuts, "coverage_ok_rank0": covered,
            "candidates_rank0": int(stats["candidates"]), "dense_tiles_rank0": int(stats["dense_tiles"]),
            "engine": engine_info,
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "pipelined": pipelined,
        "sustained": sustained,
        "hashed": hashed,
        "parity": parity,
    }
    if world > 1:
        loads = [r["bytes"] for r in ranks]
        out["ranks"] = [{k: r[k] for k in ("rank", "device", "files", "bytes", "ms_per_step", "scan_ms",
                                           "scan_frac")} for r in ranks]
        out["load_balance"] = {"max_over_mean_bytes": round(max(loads) / (sum(loads) / len(loads)), 5),
                               "max_over_mean_ms": round(max(r["ms_per_step"] for r in ranks) /
                                                         (sum(r["ms_per_step"] for r in ranks) / len(ranks)), 5)}
    if args.workload == "dedup":
        plan = dedup_plan()
        out["config"]["dedup"] = L.dedup_stability(cuts, [plan[int(i) % len(plan)] for i in idx.tolist()])
    if args.workload == "dense":
        kinds = np.array([dense_kind(int(i)) for i in idx.tolist()])
        out["config"]["adversarial_bytes_frac"] = {
            "periodic64": round(float(lens[kinds == 1].sum()) / max(span, 1), 4),
            "constant": round(float(lens[kinds == 2].sum()) / max(span, 1), 4)}
    if world == 1 and not args.no_legs:
        out["_slots"] = slots
        run_legs(args, dev_id, dbuf, offs, lens, idx, span, out)
    else:
        for h, b in slots:
            b.free()
            h.close()
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
