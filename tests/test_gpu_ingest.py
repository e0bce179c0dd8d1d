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
