"""Parity of the GPU chunk hasher (b3_kernels.hip via syncr_cdc_*_hashed) with
the BLAKE3 oracle and the official BLAKE3 vectors.

What is replaced: util::hash_binary = blake3::hash (reference src/util.rs:57-59)
per chunk in compute_file_chunks (src/protocol/file_operations.rs:757).
Bar: bit-exact 32-byte hashes, and the boundaries unchanged by hashing."""
import json
import os

import numpy as np
import pytest

import syncr_amd
from oracle import oracle as O

pytestmark = pytest.mark.gpu
M = 1 << 20
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "blake3_vectors.json")


def ref_hashes(buf, offs, cuts_per_file):
    """oracle BLAKE3 of every chunk, in fetch order."""
    o, n = [], []
    for f, cuts in zip(np.asarray(offs).tolist(), cuts_per_file):
        o += (cuts["offset"].astype(np.uint64) + np.uint64(f)).tolist()
        n += cuts["len"].astype(np.uint64).tolist()
    return O.blake3_batch(buf, np.array(o, np.uint64), np.array(n, np.uint64), nthreads=8)


def check_batch(ch, buf, offs, lens):
    got = ch.batch_arrays(buf, offs, lens, hashed=True)
    plain = ch.batch_arrays(buf, offs, lens)
    for g, p in zip(got, plain):               # hashing leaves the boundaries alone
        assert np.array_equal(g["offset"], p["offset"]) and np.array_equal(g["len"], p["len"])
    want = ref_hashes(buf, offs, got)
    have = np.concatenate([g["hash"] for g in got]) if got else np.zeros((0, 32), np.uint8)
    bad = np.nonzero((have != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {len(want)} hashes differ, first at chunk {bad[:5]}"
    return got


def test_official_vectors_one_chunk_per_file():
    """Each file is one chunk (no content cut at bits 31, no read cap): the hash
    is blake3(file) and must equal the published vector."""
    v = json.load(open(GOLDEN))
    lens = np.array([n for n, _ in v["cases"]], np.uint64)
    offs = np.zeros_like(lens)
    pad = 13                                   # unaligned file starts exercise the byte funnel
    pos = 0
    for i, n in enumerate(lens.tolist()):
        offs[i] = pos
        pos += n + pad
    buf = np.zeros(pos, np.uint8)
    for o, n in zip(offs.tolist(), lens.tolist()):
        buf[o:o + n] = (np.arange(n) % 251).astype(np.uint8)
    with syncr_amd.Chunker(31, 1 << 31, 0) as ch:
        got = ch.batch_arrays(buf, offs, lens, hashed=True)
    for (n, want), cuts in zip(v["cases"], got):
        if n == 0:
            assert cuts.size == 0              # empty file -> no chunk (chunking_test.rs:37-43)
            continue
        assert cuts.size == 1 and int(cuts["len"][0]) == n
        assert cuts["hash"][0].tobytes().hex() == want, n


# max_chunk picks the lane task: 1 leaf for a small launch whose max_chunk is at
# most 64 MiB, else 4 leaves (cdc_internal.h B3_SMALL_SPAN); bits 31 never cut
LANE_TASKS = pytest.mark.parametrize("mx", [1 << 31, 64 * M], ids=["4-leaf-tasks", "1-leaf-tasks"])


@LANE_TASKS
def test_sizes_and_alignments(mx):
    """Chunk sizes around every boundary of the decomposition (block 64 B, leaf
    1 KiB, lane 4 KiB / 1 KiB, item 256 KiB / 64 KiB, two-level tree) at all 16
    start alignments, with either lane task."""
    sizes = [1, 2, 63, 64, 65, 1023, 1024, 1025, 2047, 3073, 4095, 4096, 4097, 8193, 16383, 16384, 16385,
             65535, 65536, 65537, 131073, 262143, 262144, 262145, 524289, 1048576 + 7, 3 * M + 5]
    rng = np.random.default_rng(11)
    lens, offs, pos = [], [], 0
    for k, n in enumerate(sizes * 2):
        pos += k % 16                          # start alignment 0..15
        offs.append(pos)
        lens.append(n)
        pos += n
    buf = rng.integers(0, 256, pos, dtype=np.uint8)   # last file ends at the buffer end
    with syncr_amd.Chunker(31, mx, 0) as ch:           # one chunk per file
        got = check_batch(ch, buf, np.array(offs, np.uint64), np.array(lens, np.uint64))
    assert [int(g["len"].sum()) for g in got] == lens


@LANE_TASKS
def test_large_chunk_multi_level_tree(mx):
    """A 40 MiB chunk = 160 items of 256 KiB or 640 of 64 KiB: the tree kernel's
    batches of 64 item CVs, two or three levels."""
    n = 40 * M + 123
    buf = O.xorshift_bytes(7, n + 16)
    with syncr_amd.Chunker(31, mx, 0) as ch:
        got = ch.batch_arrays(buf, [3], [n], hashed=True)
    assert got[0].size == 1
    assert got[0]["hash"][0].tobytes() == O.blake3(buf[3:3 + n])


@pytest.mark.parametrize("bits,mx,cap", [(20, 16 * M, 2 * M), (20, 16 * M, 0), (13, 128 * 1024, 0),
                                         (8, 4096, 3000)])
def test_random_corpus_vs_oracle(bits, mx, cap):
    rng = np.random.default_rng(bits)
    lens = rng.integers(0, 3 * M, 40).astype(np.uint64)
    lens[:4] = [0, 1, 70, 5 * M]
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1] + np.arange(1, lens.size, dtype=np.uint64) * 3
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1]), dtype=np.uint8)
    with syncr_amd.Chunker(bits, mx, cap) as ch:
        check_batch(ch, buf, offs, lens)


def test_compute_file_chunks_hashes(tmp_path):
    """compute_file_chunks returns ChunkInfo{hash, offset, size} like the reference."""
    data = O.xorshift_bytes(1234, 6 * M + 99)
    p = tmp_path / "f.bin"
    p.write_bytes(data.tobytes())
    got = syncr_amd.compute_file_chunks(str(p))
    assert [c.offset + c.size for c in got] == O.chunk_production(data).tolist()
    for c in got:
        assert c.hash == O.blake3(data[c.offset:c.offset + c.size])
    assert syncr_amd.compute_file_chunks(str(p), hashed=False)[0].hash is None


def test_device_resident_zipf_corpus_hashed():
    """The full zipf10k corpus (9.73 GiB), device-resident: every chunk hash vs the oracle."""
    import bench
    sizes, idx, _ = bench.workload("zipf10k", 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    with syncr_amd.Chunker() as ch:
        buf = syncr_amd.DeviceBuffer(ch, span)
        try:
            buf.gen_corpus(offs, sizes, indices=idx)
            ch.plan(offs, sizes, span)
            ch.launch(buf.ptr, hashed=True)
            got = ch.fetch(hashed=True)
            ch.launch(buf.ptr)
            plain = ch.fetch()
            host = buf.download(span)
        finally:
            buf.free()
    for g, p in zip(got, plain):
        assert np.array_equal(g["offset"], p["offset"]) and np.array_equal(g["len"], p["len"])
    want = ref_hashes(host, offs, got)
    have = np.concatenate(got)["hash"]
    assert np.array_equal(have, want)


def test_fetch_hashed_requires_hashed_launch():
    with syncr_amd.Chunker() as ch:
        buf = syncr_amd.DeviceBuffer(ch, 4096)
        try:
            ch.plan([0], [4096], 4096)
            ch.launch(buf.ptr)
            with pytest.raises(syncr_amd.SyncrCdcError):
                ch.fetch(hashed=True)
        finally:
            buf.free()
