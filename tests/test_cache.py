"""Chunk cache (syncr_cache_*, cache.cpp): host code, runs without a GPU.

Restates the reference's ChildCache (src/cache.rs:138-260): get_chunks returns
the stored HashChunk list only when the stored mtime equals the current one
(is_valid, :167-179); set overwrites (:207-218).  Here the size must match too.
Persistence: reopening the log restores every entry; a torn tail is dropped."""
import os

import numpy as np
import pytest

import syncr_amd


def chunks(n, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, syncr_amd.CHUNK_INFO_DTYPE)
    a["len"] = rng.integers(1, 1 << 20, n)
    a["offset"] = np.concatenate([[0], np.cumsum(a["len"][:-1])])
    a["hash"] = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return a


def test_get_put_validity():
    with syncr_amd.ChunkCache() as c:
        a = chunks(5, 1)
        size = int(a["len"].sum())
        assert c.get("dir/f", 100, size) is None                    # miss
        c.put("dir/f", 100, size, a)
        got = c.get("dir/f", 100, size)
        assert np.array_equal(got, a)
        assert c.get("dir/f", 101, size) is None                    # mtime changed (cache.rs:175)
        assert c.get("dir/f", 100, size + 1) is None                # size changed
        b = chunks(3, 2)
        c.put("dir/f", 101, int(b["len"].sum()), b)                 # set overwrites
        assert np.array_equal(c.get("dir/f", 101, int(b["len"].sum())), b)
        c.put("empty", 7, 0, np.zeros(0, syncr_amd.CHUNK_INFO_DTYPE))
        assert c.get("empty", 7, 0).size == 0                        # an empty file caches []
        st = c.stats()
        assert st["entries"] == 2 and st["hits"] == 3 and st["puts"] == 3


def test_persistence_and_torn_tail(tmp_path):
    p = str(tmp_path / "chunks.cache")
    entries = {f"f{i}": chunks(i + 1, i) for i in range(20)}
    with syncr_amd.ChunkCache(p) as c:
        for k, a in entries.items():
            c.put(k, 5, int(a["len"].sum()), a)
        c.sync()
    with syncr_amd.ChunkCache(p) as c:
        for k, a in entries.items():
            assert np.array_equal(c.get(k, 5, int(a["len"].sum())), a), k
    # a crash mid-append leaves a partial record: dropped, everything before it kept
    full = os.path.getsize(p)
    with open(p, "ab") as f:
        f.write(b"\x05\x00\x00\x00abc")
    with syncr_amd.ChunkCache(p) as c:
        assert c.stats()["entries"] == len(entries)
        c.put("late", 1, 0, np.zeros(0, syncr_amd.CHUNK_INFO_DTYPE))
    with syncr_amd.ChunkCache(p) as c:
        assert c.get("late", 1, 0) is not None
        assert os.path.getsize(p) >= full


def test_refuses_foreign_file(tmp_path):
    p = tmp_path / "not_a_cache"
    p.write_bytes(b"hello world, not a cache")
    with pytest.raises(syncr_amd.SyncrCdcError):
        syncr_amd.ChunkCache(str(p))
    assert p.read_bytes() == b"hello world, not a cache"


def test_compaction_keeps_last_record(tmp_path):
    p = str(tmp_path / "c")
    with syncr_amd.ChunkCache(p) as c:
        for m in range(50):                                          # 50 overwrites of one key
            a = chunks(2, m)
            c.put("k", m, int(a["len"].sum()), a)
    with syncr_amd.ChunkCache(p) as c:
        assert c.stats()["entries"] == 1
        assert np.array_equal(c.get("k", 49, int(a["len"].sum())), a)


def test_empty_or_torn_header_file_is_a_new_cache(tmp_path):
    """a zero-length file (pre-created with touch/mkstemp, or a crash
    before the header reached the disk) and a file torn inside the magic are
    new caches, not foreign files."""
    for name, content in (("empty", b""), ("torn_magic", b"SYNC"), ("torn_header", b"SYNCRCC2\x14\x00")):
        p = tmp_path / name
        p.write_bytes(content)
        with syncr_amd.ChunkCache(str(p)) as c:
            a = chunks(3, 9)
            c.put("f", 1, int(a["len"].sum()), a)
        with syncr_amd.ChunkCache(str(p)) as c:                      # reopened: the entry survived
            assert np.array_equal(c.get("f", 1, int(a["len"].sum())), a), name


def test_old_format_log_is_a_stale_cache(tmp_path):
    """a log written by the ABI-v2 library (magic SYNCRCC1, no
    parameter header) opens as an empty cache, rewritten with the current
    header, instead of failing with EIO; its entries are never served."""
    import struct
    p = tmp_path / "old.cache"
    rec = struct.pack("<I", 1) + b"f" + struct.pack("<IQQ", 5, 100, 0)
    p.write_bytes(b"SYNCRCC1" + rec + b"\0" * 8)
    with syncr_amd.ChunkCache(str(p)) as c:
        assert c.get("f", 5, 100) is None and c.stats()["entries"] == 0
        a = chunks(2, 4)
        c.put("g", 2, int(a["len"].sum()), a)
    assert p.read_bytes()[:8] == b"SYNCRCC2"
    with syncr_amd.ChunkCache(str(p)) as c:
        assert np.array_equal(c.get("g", 2, int(a["len"].sum())), a)


def test_header_is_durable_before_first_put(tmp_path):
    p = tmp_path / "c"
    c = syncr_amd.ChunkCache(str(p))
    assert os.path.getsize(p) == 32                                  # header written + fsync'ed at open
    c.close()
    with syncr_amd.ChunkCache(str(p)) as c:
        assert c.stats()["entries"] == 0


def test_params_are_part_of_the_cache(tmp_path):
    """chunk lists cut under other chunk_bits / max_chunk / read_cap
    must never be served.  The log header records the parameters; reopening it
    under others is refused, and so is attaching it to an ingest pipeline with
    other parameters (that check runs before any device is touched)."""
    p = str(tmp_path / "c")
    with syncr_amd.ChunkCache(p, chunk_bits=20) as c:
        a = chunks(2, 3)
        c.put("f", 1, int(a["len"].sum()), a)
        got = syncr_amd.Params()
        assert syncr_amd.library().syncr_cache_get_params(c.handle, got) == 0
        assert (got.chunk_bits, got.max_chunk, got.read_cap) == (20, 16 << 20, 2 << 20)
    for kw in ({"chunk_bits": 13}, {"max_chunk": 1 << 20}, {"read_cap": 0}):
        with pytest.raises(syncr_amd.SyncrCdcError) as e:
            syncr_amd.ChunkCache(p, **kw)
        assert e.value.code == syncr_amd.E_INVAL, kw
    with syncr_amd.ChunkCache(p) as c:                               # same parameters: still valid
        assert np.array_equal(c.get("f", 1, int(a["len"].sum())), a)


def test_second_open_of_a_log_is_busy(tmp_path):
    """Two handles appending to one log would interleave records: flock."""
    p = str(tmp_path / "c")
    with syncr_amd.ChunkCache(p):
        with pytest.raises(syncr_amd.SyncrCdcError) as e:
            syncr_amd.ChunkCache(p)
        assert e.value.code == syncr_amd.E_BUSY
    with syncr_amd.ChunkCache(p):                                     # released on close
        pass


def test_failed_append_is_rolled_back(tmp_path):
    """a failed write must not leave a torn record that later puts
    append behind (they would be dropped on the next open).  RLIMIT_FSIZE makes
    the write of a big record fail part-way, in a child process."""
    import subprocess
    import sys
    p = str(tmp_path / "c")
    code = f"""
import resource, signal, numpy as np, syncr_amd
signal.signal(signal.SIGXFSZ, signal.SIG_IGN)
c = syncr_amd.ChunkCache({p!r})
small = np.zeros(1, syncr_amd.CHUNK_INFO_DTYPE); small["len"] = 5
c.put("ok", 1, 5, small)
resource.setrlimit(resource.RLIMIT_FSIZE, (4096, 4096))
big = np.zeros(200, syncr_amd.CHUNK_INFO_DTYPE); big["len"] = 1
try:
    c.put("big", 1, 200, big)
    print("NOERR")
except syncr_amd.SyncrCdcError:
    print("EIO")
try:
    c.put("after", 1, 5, small)
    print("NOERR")
except syncr_amd.SyncrCdcError:
    print("EIO")
c.close()
"""
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), timeout=120)
    assert out.stdout.split() == ["EIO", "EIO"], out.stdout + out.stderr
    with syncr_amd.ChunkCache(p) as c:                               # the log is intact up to "ok"
        assert c.get("ok", 1, 5) is not None and c.stats()["entries"] == 1
