"""Step time with `d` batches in flight (d handles, d corpus copies, round-robin launches)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np, bench, syncr_amd
sizes, idx, _ = bench.workload("zipf10k", 1)
offs = np.zeros_like(sizes); offs[1:] = np.cumsum(sizes)[:-1]; span = int(sizes.sum())
hs, bufs = [], []
for i in range(3):
    ch = syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, syncr_amd.TOKIO_READ_CAP)
    b = syncr_amd.DeviceBuffer(ch, span); b.gen_corpus(offs, sizes, indices=idx)
    ch.plan(offs, sizes, span); hs.append(ch); bufs.append(b)
hashed = "--hashed" in sys.argv
for rnd in range(3):
    for d in (1, 2, 3):
        for k in range(2 * d):
            hs[k % d].launch(bufs[k % d].ptr, hashed=hashed)
        for h in hs: h.synchronize()
        K = 30
        t0 = time.perf_counter()
        for k in range(K):
            hs[k % d].launch(bufs[k % d].ptr, hashed=hashed)
        for h in hs: h.synchronize()
        dt = (time.perf_counter() - t0) / K
        print(f"round {rnd} depth {d}: {dt*1e3:.4f} ms/step  {span/dt/2**30:.1f} GiB/s", flush=True)
ref = hs[0].fetch(hashed=hashed)
for h in hs[1:]:
    got = h.fetch(hashed=hashed)
    assert all(np.array_equal(a, b) for a, b in zip(ref, got))
print("results identical across slots")
