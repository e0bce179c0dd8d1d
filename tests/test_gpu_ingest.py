"""Batched ingest pipeline (syncr_ingest_*, ingest.cpp) vs the CPU oracle.

Replaces traverse_and_stream's serial per-file loop (reference
src/protocol/file_operations.rs:544-715, :599-605).  Per file, in submission
order: the ChunkInfo list (offset, size, BLAKE3) of compute_file_chunks
(:721-788), or an empty list with an error status for an unreadable file
(:727-744).  Bar: bit-exact boundaries and hashes."""
import errno

import numpy as np
import pytest

import syncr_amd
from oracle import oracle as O

pytestmark = pytest.mark.gpu
M = 1 << 20


def expect(data, bits=20, mx=16 * M, cap=2 * M):
    ends = (O.chunk_production(data, bits, mx, cap) if cap else O.chunk_ideal(data, bits, mx)).astype(np.uint64)
    starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)[:ends.size]
    lens = ends - starts
    hs = O.blake3_batch(data, starts, lens, nthreads=8) if ends.size else np.zeros((0, 32), np.uint8)
    return starts, lens, hs


def check(res, files, **kw):
    assert [t for t, _, _ in res] == list(range(len(files)))        # submission order
    for (tag, status, got), data in zip(res, files):
        assert status == 0, tag
        starts, lens, hs = expect(data, **kw)
        assert np.array_equal(got["offset"], starts), tag
        assert np.array_equal(got["len"].astype(np.uint64), lens), tag
        assert np.array_equal(got["hash"], hs), tag


def corpus(n, seed, maxlen):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, n)
    lens[:3] = [0, 1, maxlen + 3 * M]           # empty, tiny, bigger than a batch
    return [O.xorshift_bytes(seed * 1000 + i, int(m)) for i, m in enumerate(lens)]


@pytest.mark.parametrize("depth", [1, 3])
def test_bytes_many_batches(depth):
    files = corpus(60, 3, 3 * M)
    with syncr_amd.Ingest(batch_bytes=4 * M, depth=depth, copy_threads=4) as g:
        for i, f in enumerate(files):
            g.submit(f, i)
        g.flush()
        st = g.stats()
        res = g.results
    assert st["files"] == len(files) and st["bytes"] == sum(f.size for f in files) and st["batches"] > 5
    check(res, files)


def test_files_and_errors(tmp_path):
    files = corpus(25, 5, 5 * M)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    paths.insert(7, str(tmp_path / "missing.bin"))          # file_operations.rs:727-733
    got = []
    with syncr_amd.Ingest(batch_bytes=8 * M, depth=2, copy_threads=4,
                          on_file=lambda t, s, a: got.append((t, s, a))) as g:
        for i, p in enumerate(paths):
            g.submit_file(p, i)
        g.flush()
    assert got[7][1] == -errno.ENOENT and got[7][2].size == 0
    del got[7]
    check([(i, s, a) for i, (_, s, a) in enumerate(got)], files)


def test_reserve_commit_ideal_semantics():
    files = corpus(20, 9, 2 * M)
    with syncr_amd.Ingest(13, 128 * 1024, 0, batch_bytes=2 * M, depth=2) as g:
        for i, f in enumerate(files):
            dst = g.reserve(f.size)
            dst[:] = f
            g.commit(i)
        g.flush()
        res = g.results
    check(res, files, bits=13, mx=128 * 1024, cap=0)


def test_flush_is_repeatable():
    files = corpus(8, 11, M)
    with syncr_amd.Ingest(batch_bytes=2 * M, depth=2) as g:
        for i, f in enumerate(files[:4]):
            g.submit(f, i)
        g.flush()
        for i, f in enumerate(files[4:], 4):
            g.submit(f, i)
        g.flush()
        g.flush()
        res = g.results
    check(res, files)


def test_chunk_cache_skips_unchanged_files(tmp_path):
    """src/cache.rs:183-203 wired into the walk: a second pass over unchanged
    files is served from the cache (identical ChunkInfo lists); a modified file
    (new mtime) is re-chunked; the cache persists across handles."""
    import os
    files = corpus(12, 13, 3 * M)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    cpath = str(tmp_path / "chunks.cache")

    def run(cache):
        res = []
        with syncr_amd.Ingest(batch_bytes=4 * M, depth=2, cache=cache,
                              on_file=lambda t, s, a: res.append((t, s, a))) as g:
            for i, p in enumerate(paths):
                g.submit_file(p, i)
            g.flush()
            return res, g.stats()

    with syncr_amd.ChunkCache(cpath) as c:
        first, st1 = run(c)
        assert st1["cache_hits"] == 0
        check(first, files)
        second, st2 = run(c)
        assert st2["cache_hits"] == len(files) and st2["bytes"] == 0
        for (t1, s1, a1), (t2, s2, a2) in zip(first, second):
            assert t1 == t2 and s1 == s2 and np.array_equal(a1, a2)
    # modify one file (content and mtime): only it is re-chunked
    new = O.xorshift_bytes(777, 2 * M + 5)
    with open(paths[4], "wb") as fh:
        fh.write(new.tobytes())
    st = os.stat(paths[4])
    os.utime(paths[4], (st.st_atime, st.st_mtime + 10))
    files[4] = new
    with syncr_amd.ChunkCache(cpath) as c:                   # reopened from disk
        third, st3 = run(c)
    assert st3["cache_hits"] == len(files) - 1
    check(third, files)


# ---- one pipeline over several devices (syncr_ingest_open_multi) ----------
# The pool's box has one GPU, so "two devices" are two sub-pipelines on device
# 0: the same code path (one worker thread, handles and streams per listed
# device, LPT assignment, reordering) as on an 8-GPU node.

@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_device_bytes_in_submission_order(devices):
    files = corpus(90, 21, 3 * M)
    with syncr_amd.Ingest(batch_bytes=4 * M, depth=2, copy_threads=4, devices=devices) as g:
        for i, f in enumerate(files):
            g.submit(f, 1000 + i)
        g.flush()
        st, per = g.stats(), g.device_stats()
        res = g.results
    assert [t for t, _, _ in res] == [1000 + i for i in range(len(files))]
    check([(t - 1000, s, a) for t, s, a in res], files)
    assert st["files"] == len(files) and st["bytes"] == sum(f.size for f in files)
    assert len(per) == len(devices) and all(p["device"] == 0 for p in per)
    assert sum(p["files"] for p in per) == len(files) and all(p["files"] > 0 for p in per)
    loads = [p["bytes"] for p in per]                        # online LPT: within one file of the mean
    assert max(loads) - min(loads) <= max(f.size for f in files)


def test_multi_device_files_errors_and_cache(tmp_path):
    """submit_file on two sub-pipelines: missing files keep their place in the
    order with -ENOENT; a cache attached to the multi pipeline serves the
    second pass from every sub-pipeline."""
    files = corpus(30, 23, 4 * M)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    paths.insert(5, str(tmp_path / "missing.bin"))
    cpath = str(tmp_path / "c.cache")

    def run(cache):
        got = []
        with syncr_amd.Ingest(batch_bytes=6 * M, depth=2, copy_threads=4, devices=[0, 0], cache=cache,
                              on_file=lambda t, s, a: got.append((t, s, a))) as g:
            for i, p in enumerate(paths):
                g.submit_file(p, i)
            g.flush()
            return got, g.stats()

    with syncr_amd.ChunkCache(cpath) as c:
        first, st1 = run(c)
        second, st2 = run(c)
    for got in (first, second):
        assert [t for t, _, _ in got] == list(range(len(paths)))
        assert got[5][1] == -errno.ENOENT and got[5][2].size == 0
        rest = [x for k, x in enumerate(got) if k != 5]
        check([(i, s, a) for i, (_, s, a) in enumerate(rest)], files)
    assert st1["cache_hits"] == 0 and st2["cache_hits"] == len(files)


def test_multi_device_reserve_commit_zipf_subset():
    """A Zipf-sized subset (SURVEY §8d config 3 sizes, the 300 smallest plus the
    largest files up to 512 MiB in total) through reserve/commit on two
    sub-pipelines: every boundary and BLAKE3 bit-exact vs the oracle."""
    import bench
    sizes = bench.zipf_sizes()
    order = np.argsort(sizes, kind="stable")
    pick = list(order[:300])
    tot = int(sizes[pick].sum())
    for i in order[::-1]:
        if tot + int(sizes[i]) > 512 * M:
            continue
        pick.append(i)
        tot += int(sizes[i])
        if tot > 480 * M:
            break
    pick = sorted(int(i) for i in pick)
    files = [O.corpus_fill(np.array([sizes[i]], np.uint64), first_index=i)[0] for i in pick]
    with syncr_amd.Ingest(batch_bytes=64 * M, depth=2, copy_threads=8, devices=[0, 0]) as g:
        for k, f in enumerate(files):
            dst = g.reserve(f.size)
            dst[:] = f
            g.commit(k)
        g.flush()
        res = g.results
    check(res, files)


def test_multi_device_state_errors():
    with syncr_amd.Ingest(batch_bytes=M, depth=1, devices=[0, 0]) as g:
        g.reserve(10)
        with pytest.raises(syncr_amd.SyncrCdcError):
            g.submit(np.zeros(5, np.uint8), 1)               # reserve outstanding
        with pytest.raises(syncr_amd.SyncrCdcError):
            g.flush()
        g.commit(0)
        g.flush()
        assert [t for t, _, _ in g.results] == [0]


def test_first_read_failure_is_empty(tmp_path):
    """A directory opens but its first read fails (EISDIR): compute_file_chunks
    warns and returns an empty list (file_operations.rs:738-743); the pipeline
    reports -EISDIR with no chunks and keeps the order of the other files."""
    files = corpus(6, 29, 2 * M)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    d = tmp_path / "subdir"
    d.mkdir()
    paths.insert(2, str(d))
    for devices in (None, [0, 0]):
        got = []
        with syncr_amd.Ingest(batch_bytes=4 * M, depth=2, devices=devices,
                              on_file=lambda t, s, a: got.append((t, s, a))) as g:
            for i, p in enumerate(paths):
                g.submit_file(p, i)
            g.flush()
        assert [t for t, _, _ in got] == list(range(len(paths)))
        assert got[2][1] == -errno.EISDIR and got[2][2].size == 0
        check([(i, s, a) for i, (_, s, a) in enumerate(got[:2] + got[3:])], files)


def test_periodic_files_split_walks():
    """Low-entropy input through the pipeline: bits-20 periodic files (a cut
    every 64 bytes) of up to 6 MiB between random ones.  A slot's handle turns
    on split walks once a batch of it held many candidates,
    so later batches walk split; every ChunkInfo (boundaries + BLAKE3) must
    still equal the oracle's, in submission order."""
    import bench
    pat = bench.periodic_pattern()
    rng = np.random.default_rng(31)
    files = []
    for i in range(24):
        n = int(rng.integers(300 << 10, 6 * M))
        files.append(np.resize(pat, n) if i % 2 == 0 else O.xorshift_bytes(7000 + i, n))
    with syncr_amd.Ingest(batch_bytes=8 * M, depth=2, copy_threads=4) as g:
        for i, f in enumerate(files):
            g.submit(f, i)
        g.flush()
        res = g.results
    assert [t for t, _, _ in res] == list(range(len(files)))
    for (tag, status, got), data in zip(res, files):
        assert status == 0, tag
        ends = O.chunk_production_window(data, 20, 16 * M, 2 * M).astype(np.uint64)
        starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)[:ends.size]
        assert np.array_equal(got["offset"], starts), tag
        assert np.array_equal(got["len"].astype(np.uint64), ends - starts), tag
        hs = O.blake3_batch(data, starts, ends - starts, nthreads=8)
        assert np.array_equal(got["hash"], hs), tag


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_oversized_file_fails_alone(tmp_path, devices):
    """a file whose batch cannot be allocated (here a
    sparse 512 GiB file: more than the GPU's memory) fails by itself.
    Single device: submit_file raises ENOMEM for that call.  Multi-device: the
    call returned before the job ran, so the file is delivered in its place
    with -ENOMEM and no chunks; either way every later file is still chunked
    and delivered in order and flush succeeds (only engine errors are sticky)."""
    files = corpus(8, 41, 2 * M)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    big = tmp_path / "sparse.bin"
    try:
        with open(big, "wb") as fh:
            fh.truncate(512 << 30)
    except OSError:
        pytest.skip("no sparse files here")
    paths.insert(3, str(big))
    got = []
    with syncr_amd.Ingest(batch_bytes=4 * M, depth=2, copy_threads=2, devices=devices,
                          on_file=lambda t, s, a: got.append((t, s, a))) as g:
        for i, p in enumerate(paths):
            if devices is None and i == 3:
                with pytest.raises(syncr_amd.SyncrCdcError) as ei:
                    g.submit_file(p, i)
                assert ei.value.code == -errno.ENOMEM
                continue
            g.submit_file(p, i)
        g.flush()
    if devices is None:
        assert [t for t, _, _ in got] == [i for i in range(len(paths)) if i != 3]
        rest = got
    else:
        assert [t for t, _, _ in got] == list(range(len(paths)))
        assert got[3][1] == -errno.ENOMEM and got[3][2].size == 0
        rest = got[:3] + got[4:]
    check([(i, s, a) for i, (_, s, a) in enumerate(rest)], files)


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_read_fault_keeps_reference_prefix(tmp_path, devices):
    """the read-error contract end to end, through an injected read
    fault (syncr_ingest_set_read_fault).  A read that fails at file offset P > 0
    keeps the chunks compute_file_chunks cut before its loop breaks
    (file_operations.rs:776-782; oracle orc_chunk_production_read_error) and
    reports -errno; P = 0 is the failed first read (:738-743): -errno, no
    chunks; a fault with errno 0 is EOF at P (a file that shrank): status 0 and
    the chunks of the P bytes read.  Faults mid-piece, on a 2 MiB read-piece
    boundary, near a cut and past the end; boundaries and BLAKE3 bit-exact."""
    import bench
    data = O.xorshift_bytes(4242, 13 * M + 777)
    periodic = np.resize(bench.periodic_pattern(), M + 3)   # small: the literal oracle memmoves per cut
    p_rand, p_per = tmp_path / "rand.bin", tmp_path / "per.bin"
    p_rand.write_bytes(data.tobytes())
    p_per.write_bytes(periodic.tobytes())
    ends = O.chunk_production(data)
    cases = [(p_rand, data, 5 * M + 123, errno.EIO), (p_rand, data, 6 * M, errno.EIO),
             (p_rand, data, int(ends[2]) + 1, errno.EIO), (p_rand, data, 0, errno.EIO),
             (p_rand, data, 7 * M + 5, 0), (p_rand, data, 20 * M, errno.EIO),
             (p_per, periodic, 700 * 1024 + 17, errno.EIO), (p_per, periodic, 512 * 1024 + 64, 0)]
    got = []
    with syncr_amd.Ingest(batch_bytes=16 * M, depth=2, copy_threads=4, devices=devices,
                          on_file=lambda t, s, a: got.append((t, s, a))) as g:
        for i, (path, _, P, err) in enumerate(cases):
            g.set_read_fault(P, err)
            g.submit_file(str(path), i)
            g.flush()
        g.set_read_fault(None)
        g.submit_file(str(p_rand), len(cases))
        g.flush()
    assert [t for t, _, _ in got] == list(range(len(cases) + 1))
    for (tag, status, arr), (_, d, P, err) in zip(got, cases + [(p_rand, data, data.size, 0)]):
        if P >= d.size:                                    # the fault lies past the end: a complete read
            want_status, e = 0, O.chunk_production_window(d)
        elif err:
            want_status, e = -err, O.chunk_production_read_error(d, P)
        else:
            want_status, e = 0, O.chunk_production_window(d[:P])
        assert status == want_status, (tag, status, want_status)
        e = e.astype(np.uint64)
        starts = np.concatenate([[0], e[:-1]]).astype(np.uint64)[:e.size]
        assert np.array_equal(arr["offset"], starts), tag
        assert np.array_equal(arr["len"].astype(np.uint64), e - starts), tag
        hs = O.blake3_batch(d, starts, e - starts, nthreads=8) if e.size else np.zeros((0, 32), np.uint8)
        assert np.array_equal(arr["hash"], hs), tag


FD_CHILD = r'''
import json, os, resource, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import syncr_amd
from oracle import oracle as O
paths = sys.argv[2:]
res = {}
with syncr_amd.Ingest(batch_bytes=64 << 20, depth=2, copy_threads=2,
                      on_file=lambda t, st, a: res.__setitem__(t, (st, a))) as g:
    open_now = len(os.listdir("/proc/self/fd"))
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    lim = open_now + 80                     # the pipeline's 64 open reads + headroom, far below len(paths)
    resource.setrlimit(resource.RLIMIT_NOFILE, (lim, hard))
    for i, p in enumerate(paths):
        g.submit_file(p, i)
    g.flush()
bad = 0
for i, p in enumerate(paths):
    st, a = res[i]
    data = np.fromfile(p, np.uint8)
    ends = O.chunk_production(data)
    got = (a["offset"].astype(np.uint64) + a["len"].astype(np.uint64))
    bad += st != 0 or not np.array_equal(got, ends.astype(np.uint64))
print(json.dumps({"files": len(paths), "bad": int(bad), "limit": lim,
                  "statuses": sorted({int(res[i][0]) for i in range(len(paths))})}))
'''


def test_submit_file_bounded_open_files(tmp_path):
    """submit_file keeps a file's descriptor until its reads finish;
    with reads queued faster than one pool thread serves them, the open files
    are capped (MAX_OPEN_READS = 64 per pipeline: submit_file helps with the
    queued reads or waits), so 3000 files go through a process whose descriptor
    limit is 80 above what it has open, each with status 0 and the oracle's
    cuts -- the reference opens one file at a time (file_operations.rs:599-605)
    and lists every file."""
    import json
    import os
    import subprocess
    import sys
    rng = np.random.default_rng(11)
    paths = []
    for i in range(3000):
        p = tmp_path / f"f{i:05d}"
        p.write_bytes(O.xorshift_bytes(7000 + i, int(rng.integers(1, 24 << 10))).tobytes())
        paths.append(str(p))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", FD_CHILD, root, *paths], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["files"] == 3000 and out["bad"] == 0 and out["statuses"] == [0], out
