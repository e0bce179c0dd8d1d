"""Step time with no timing events, scan-only events and every-phase events (one process)."""
import os, sys, time, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np, bench, syncr_amd
sizes, idx, _ = bench.workload("zipf10k", 1)
offs = np.zeros_like(sizes); offs[1:] = np.cumsum(sizes)[:-1]; span = int(sizes.sum())
ch = syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, syncr_amd.TOKIO_READ_CAP)
b = syncr_amd.DeviceBuffer(ch, span); b.gen_corpus(offs, sizes, indices=idx); ch.plan(offs, sizes, span)
for _ in range(5): ch.launch(b.ptr)
ch.synchronize()
res = {m: [] for m in ("none", "scan", "all")}
for rnd in range(5):
    for m in res:
        ch.set_timing(m != "none", scan_only=(m == "scan"))
        t0 = time.perf_counter()
        for _ in range(20): ch.launch(b.ptr)
        ch.synchronize()
        res[m].append((time.perf_counter() - t0) / 20 * 1e3)
        ch.set_timing(False)
for m, v in res.items():
    print(f"{m:5s} step med {statistics.median(v):.4f} ms  min {min(v):.4f}")
