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
