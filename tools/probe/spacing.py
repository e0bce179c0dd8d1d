import sys, time, statistics, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, bench, syncr_amd
sizes, idx, _ = bench.workload("zipf10k", 1)
read_cap = syncr_amd.TOKIO_READ_CAP
offs = np.zeros_like(sizes); offs[1:] = np.cumsum(sizes)[:-1]; span = int(sizes.sum())
ch = syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, read_cap); buf = syncr_amd.DeviceBuffer(ch, span); buf.gen_corpus(offs, sizes, indices=idx)
ch.plan(offs, sizes, span)
for _ in range(3): ch.launch(buf.ptr)
ch.synchronize()
for burst in (1, 2, 5, 20, 50):
    res = []
    for rep in range(3):
        ch.synchronize(); time.sleep(0.05)
        ch.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(burst): ch.launch(buf.ptr)
        ch.synchronize()
        dt = (time.perf_counter() - t0) / burst
        ms, n = ch.kernel_times(); ch.set_timing(False)
        res.append((ms[0] / n, dt * 1e3))
    print("burst %3d: scan %.4f ms  step %.4f ms" % (burst, statistics.median(r[0] for r in res), statistics.median(r[1] for r in res)), flush=True)
