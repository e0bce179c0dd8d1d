"""Parity of the HIP engine (libsyncr_cdc.so via the C ABI) with the CPU oracle.

Bar: bit-exact cut offsets and counts (integer work).  Every test here runs the
HIP kernels on the GPU; the oracle is only the checker."""
import numpy as np
import pytest

import syncr_amd
from golden_inputs import make_input
from oracle import oracle as O

pytestmark = pytest.mark.gpu
M = 1 << 20


def ends_of(cuts: np.ndarray) -> list:
    return (cuts["offset"].astype(np.uint64) + cuts["len"].astype(np.uint64)).tolist()


def check_contiguous(cuts, n, mx):
    off = 0
    for o, ln, _ in cuts.tolist():
        assert o == off and 1 <= ln <= mx
        off += ln
    assert off == n


def oracle_ends(data, bits, mx, cap):
    return (O.chunk_production(data, bits, mx, cap) if cap else O.chunk_ideal(data, bits, mx)).tolist()


# --------------------------------------------------------------------------
def test_golden_kats(kat_cases, chunkers):
    for c in kat_cases:
        data = make_input(c["recipe"])
        ch = chunkers(c["chunk_bits"], c["max_chunk"], c["read_cap"])
        cuts = ch.cut_array(data)
        assert ends_of(cuts) == c["ends"], c["name"]
        check_contiguous(cuts, data.size, c["max_chunk"])


def test_reference_small_and_empty(chunkers):
    ch = chunkers()
    assert [(c.offset, c.size) for c in ch.chunk_bytes(b"small")] == [(0, 5)]   # protocol_list_test.rs:305-322
    assert ch.chunk_bytes(b"") == []                                           # chunking_test.rs:37-43
    assert syncr_amd.chunk_data(b"Small file") == [(0, 10)]                    # chunking_test.rs:26-34


def test_compute_file_chunks_file(tmp_path, chunkers):
    data = O.xorshift_bytes(99, 5 * M + 17)
    p = tmp_path / "f.bin"
    p.write_bytes(data.tobytes())
    got = syncr_amd.compute_file_chunks(str(p), chunkers())
    assert [c.offset + c.size for c in got] == O.chunk_production(data).tolist()


def test_device_generator_matches_cpu(chunkers):
    ch = chunkers()
    lens = np.array([1, 4095, 4096, 4097, 0, 65536 + 3, 3 * M + 5, 77], np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    total = int(lens.sum())
    buf = syncr_amd.DeviceBuffer(ch, total + 64)
    try:
        idx = np.array([5, 9, 2, 100000, 3, 17, 8, 12345], np.uint64)
        buf.gen_corpus(offs, lens, indices=idx)
        dev = buf.download(total)
        for i in range(lens.size):
            ref = O.xorshift_bytes(O.corpus_seed(int(idx[i])), int(lens[i]), discard=64)
            assert np.array_equal(dev[int(offs[i]): int(offs[i] + lens[i])], ref), i
    finally:
        buf.free()


def _batch_vs_oracle(ch, buf, offs, lens, bits, mx, cap):
    res = ch.batch_arrays(buf, offs, lens)
    for i, (o, n) in enumerate(zip(np.asarray(offs).tolist(), np.asarray(lens).tolist())):
        f = buf[o: o + n]
        assert ends_of(res[i]) == oracle_ends(f, bits, mx, cap), (i, o, n, bits, mx, cap)
        assert (res[i]["file"] == i).all()


@pytest.mark.parametrize("bits,mx,cap", [(20, 16 << 20, 2 << 20), (20, 16 << 20, 0), (13, 1 << 17, 0),
                                         (13, 1 << 17, 65536), (8, 4096, 0), (16, 1 << 18, 5000),
                                         (17, 1 << 19, 0), (31, 1 << 20, 0), (1, 100, 0), (4, 50, 7)])
def test_many_small_files(chunkers, bits, mx, cap):
    """Edge sizes: 0, 1, 62..66 bytes, run/tile boundaries (144 / 18432), odd offsets."""
    rng = np.random.default_rng(bits * 1000 + cap)
    sizes = [0, 1, 2, 62, 63, 64, 65, 66, 143, 144, 145, 18431, 18432, 18433, 36863, 100000, 0, 7]
    sizes += rng.integers(0, 60000, 120).tolist()
    lens = np.array(sizes, np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    data[: data.size // 3] &= 7                         # some low-entropy regions
    _batch_vs_oracle(chunkers(bits, mx, cap), data, offs, lens, bits, mx, cap)


def test_quarter_million_tiny_files_hashed():
    """A plan whose tables exceed the pinned staging group limit (4 MiB: the
    synchronous-copy path, its counter block zeroed by a memset): 250 000 files
    of 0..40 bytes (a few hold a head hit), hashed; every file's cuts and every
    chunk's BLAKE3 against the oracle."""
    rng = np.random.default_rng(250)
    lens = rng.integers(0, 41, 250_000).astype(np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    data = rng.integers(0, 256, max(int(lens.sum()), 1), dtype=np.uint8)
    with syncr_amd.Chunker() as ch:
        d = syncr_amd.DeviceBuffer(ch, data.size)
        try:
            d.upload(data)
            ch.plan(offs, lens, int(lens.sum()))
            ch.launch(d.ptr, hashed=True)
            got = ch.fetch(hashed=True)
        finally:
            d.free()
    want = O.chunk_batch(data, offs, lens)
    assert len(got) == lens.size
    bad = [i for i in range(lens.size) if ends_of(got[i]) != want[i].tolist()]
    assert not bad, (len(bad), bad[:5])
    co = np.concatenate([offs[i] + got[i]["offset"].astype(np.uint64) for i in range(lens.size)])
    cl = np.concatenate([got[i]["len"].astype(np.uint64) for i in range(lens.size)])
    hs = np.concatenate([got[i]["hash"] for i in range(lens.size)])
    assert np.array_equal(hs, O.blake3_batch(data, co, cl, nthreads=8))


def test_gaps_and_unsorted_table(chunkers):
    """Files with holes between them and a table not sorted by offset."""
    rng = np.random.default_rng(7)
    n = 60
    lens = rng.integers(0, 300000, n).astype(np.uint64)
    gaps = rng.integers(0, 5000, n).astype(np.uint64)
    offs = np.zeros(n, np.uint64)
    acc = 0
    for i in range(n):
        acc += int(gaps[i])
        offs[i] = acc
        acc += int(lens[i])
    data = rng.integers(0, 256, acc + 100, dtype=np.uint8)
    perm = rng.permutation(n)
    for bits, mx, cap in ((20, 16 << 20, 2 << 20), (12, 1 << 15, 0)):
        _batch_vs_oracle(chunkers(bits, mx, cap), data, offs[perm], lens[perm], bits, mx, cap)


def test_dense_tiles_low_entropy(chunkers):
    """Data with >64 candidates per 18 KiB tile goes through the dense-bitmap path."""
    data = O.xorshift_bytes(4242, 2 * M)
    data = (data & 1).astype(np.uint8)
    for bits, mx, cap in ((6, 4096, 0), (8, 1 << 12, 3000), (10, 1 << 14, 0)):
        ch = chunkers(bits, mx, cap)
        cuts = ch.cut_array(data)
        assert ends_of(cuts) == oracle_ends(data, bits, mx, cap)


def test_periodic_pattern_every_64(chunkers):
    """A 64-byte period whose window hits: one G-candidate every 64 bytes."""
    bits = 12
    rng = np.random.default_rng(3)
    for _ in range(2000):
        pat = rng.integers(0, 256, 64, dtype=np.uint8)
        rep = np.tile(pat, 2)
        if O.chunk_ideal(rep, bits, 1 << 20).tolist() != [128]:
            break
    data = np.tile(pat, 40000)
    for cap in (0, 1 << 16):
        ch = chunkers(bits, 1 << 16, cap)
        assert ends_of(ch.cut_array(data)) == oracle_ends(data, bits, 1 << 16, cap)


def test_dense_workload_subset(chunkers):
    """bench.py --workload dense at test size: files that are the bits-20
    periodic pattern (a cut every 64 bytes: dense tiles, candidate-array and
    cut-capacity overflow re-runs, long chained resolve walks), constant-byte
    files (MAX / read-cap cuts) and random files, packed back to back at
    unaligned offsets, in both semantics; every cut bit-exact vs the oracle."""
    import bench
    pat = bench.periodic_pattern()
    rng = np.random.default_rng(77)
    files = []
    for i in range(24):
        n = int(rng.integers(0, 5 * M)) if i % 5 else int(rng.integers(0, 300))
        k = i % 3
        files.append(np.resize(pat, n) if k == 0 else
                     (np.full(n, i, np.uint8) if k == 1 else O.xorshift_bytes(900 + i, n)))
    files.append(np.resize(pat, 18 * M + 13))                  # > MAX: forced cut, then saturated walk
    lens = np.array([f.size for f in files], np.uint64)
    gaps = rng.integers(0, 40, lens.size).astype(np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens + gaps)[:-1]
    span = int(offs[-1] + lens[-1]) + 5
    data = np.zeros(span, np.uint8)
    for o, f in zip(offs.tolist(), files):
        data[o:o + f.size] = f
    for cap in (2 << 20, 0):
        res = chunkers(20, 16 << 20, cap).batch_arrays(data, offs, lens)
        for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
            # the literal loop without copy_within (O(n) per 64-byte chunk here)
            want = (O.chunk_production_window(data[o:o + n], 20, 16 << 20, cap) if cap
                    else O.chunk_ideal(data[o:o + n], 20, 16 << 20)).tolist()
            assert ends_of(res[i]) == want, (i, n, cap)


def test_error_contract(chunkers):
    import ctypes
    L = syncr_amd.library()
    ch = chunkers()
    h = ch.handle
    # launch before plan -> ESTATE on a fresh handle
    fresh = syncr_amd.Chunker()
    assert L.syncr_cdc_launch(fresh.handle, None, None) == -71
    fresh.close()
    # overlapping files -> EINVAL
    offs = np.array([0, 10], np.uint64)
    lens = np.array([20, 20], np.uint64)
    assert L.syncr_cdc_plan(h, offs.ctypes.data, lens.ctypes.data, 2, 100) == -22
    # file beyond span -> EINVAL
    assert L.syncr_cdc_plan(h, offs.ctypes.data, lens.ctypes.data, 1, 10) == -22
    # capacity too small -> ERANGE with the needed count
    data = O.xorshift_bytes(5, 8 * M)
    out = np.zeros(2, syncr_amd.CUT_DTYPE)
    n = ctypes.c_uint64(0)
    rc = L.syncr_cdc_chunk_host(h, data.ctypes.data, data.size, out.ctypes.data, 2, ctypes.byref(n))
    assert rc == -34 and n.value == len(O.chunk_production(data))
    # unaligned device pointer -> EINVAL
    buf = syncr_amd.DeviceBuffer(ch, 4096)
    ch.plan([0], [100], 100)
    assert L.syncr_cdc_launch(h, buf.ptr + 1, None) == -22
    buf.free()


def test_uniform_corpus_device_resident(chunkers, uniform_corpus_golden):
    """SURVEY §8d config 2 at full size (1 GiB), generated and chunked on the device."""
    g = uniform_corpus_golden
    ch = chunkers()
    lens = np.full(g["files"], g["file_len"], np.uint64)
    offs = np.arange(g["files"], dtype=np.uint64) * np.uint64(g["file_len"])
    buf = syncr_amd.DeviceBuffer(ch, int(lens.sum()))
    try:
        buf.gen_corpus(offs, lens)
        ch.plan(offs, lens, int(lens.sum()))
        for _ in range(2):                      # repeated launches give identical results
            ch.launch(buf.ptr)
            res = ch.fetch()
            assert [ends_of(r) for r in res] == g["ends"]
    finally:
        buf.free()


def zipf_sizes(n=10000, seed=20251212):
    z = np.random.default_rng(seed).zipf(1.5, n).astype(np.float64)
    return np.minimum(4096.0 * z, float(128 * M)).astype(np.uint64)


@pytest.mark.slow
def test_zipf_corpus_full_size(chunkers):
    """SURVEY §8d config 3 (10 000 Zipf files, 9.73 GiB) at full size: every
    file's cuts vs the oracle in both modes."""
    lens = zipf_sizes()
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    span = int(lens.sum())
    assert abs(span / 2**30 - 9.73) < 0.02
    for cap in (2 << 20, 0):
        ch = chunkers(20, 16 << 20, cap)
        buf = syncr_amd.DeviceBuffer(ch, span)
        try:
            buf.gen_corpus(offs, lens)
            ch.plan(offs, lens, span)
            ch.launch(buf.ptr)
            res = ch.fetch()
            host = buf.download(span)
        finally:
            buf.free()
        ref = O.chunk_batch(host, offs, lens, read_cap=cap,
                            mode=O.MODE_PRODUCTION if cap else O.MODE_IDEAL)
        bad = [i for i in range(lens.size) if ends_of(res[i]) != ref[i].tolist()]
        assert not bad, bad[:10]
        del host


@pytest.mark.slow
def test_single_file_over_4gib(chunkers):
    """One 5 GiB file (the reference's offsets are u64: file_operations.rs:721-788):
    the resolve walk's 64-bit path, cut offsets past 2^32 and the hash kernels'
    64-bit chunk starts, in both modes, vs the oracle; hashes vs the BLAKE3 oracle."""
    n = 5 << 30
    lens = np.array([n], np.uint64)
    offs = np.zeros(1, np.uint64)
    for cap in (2 << 20, 0):
        ch = chunkers(20, 16 << 20, cap)
        buf = syncr_amd.DeviceBuffer(ch, n)
        try:
            buf.gen_corpus(offs, lens)
            ch.plan(offs, lens, n)
            ch.launch(buf.ptr, hashed=True)
            res = ch.fetch(hashed=True)[0]
            host = buf.download(n)
        finally:
            buf.free()
        ref = O.chunk_batch(host, offs, lens, read_cap=cap,
                            mode=O.MODE_PRODUCTION if cap else O.MODE_IDEAL)[0]
        assert ends_of(res) == ref.tolist()
        assert int(res["offset"][-1]) > (1 << 32)
        want = O.blake3_batch(host, res["offset"].astype(np.uint64), res["len"].astype(np.uint64), nthreads=8)
        assert np.array_equal(res["hash"], want)
        del host


@pytest.mark.slow
def test_dedup_corpus(chunkers):
    """SURVEY §8d config 5 (scaled to 200 variants of a 32 MiB base): bit-exact
    and boundary-stable (most base cuts survive a small edit, shift-adjusted)."""
    rng = np.random.default_rng(55)
    base = O.xorshift_bytes(31337, 32 * M)
    files, edits = [], []
    for _ in range(200):
        pos = int(rng.integers(0, base.size))
        ln = int(rng.integers(1, 257))
        kind = rng.choice(["overwrite", "overwrite", "insert", "delete"])
        ins = rng.integers(0, 256, ln, dtype=np.uint8)
        if kind == "overwrite":
            f = base.copy(); f[pos:pos + ln] = ins[: max(0, min(ln, base.size - pos))]
            delta = 0
        elif kind == "insert":
            f = np.concatenate([base[:pos], ins, base[pos:]]); delta = ln
        else:
            f = np.concatenate([base[:pos], base[pos + ln:]]); delta = -min(ln, base.size - pos)
        files.append(f); edits.append((pos, delta))
    lens = np.array([f.size for f in files], np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    buf = np.concatenate(files)
    ch = chunkers()
    res = ch.batch_arrays(buf, offs, lens)
    ref = O.chunk_batch(buf, offs, lens)
    base_cuts = set(O.chunk_production(base).tolist())
    kept = []
    for i in range(len(files)):
        assert ends_of(res[i]) == ref[i].tolist(), i
        pos, delta = edits[i]
        adj = {e - delta if e > pos else e for e in ends_of(res[i])}
        kept.append(len(adj & base_cuts) / len(base_cuts))
    assert np.median(kept) >= 0.9


def test_kernel_timing_api(chunkers):
    ch = chunkers()
    data_len = 64 * M
    buf = syncr_amd.DeviceBuffer(ch, data_len)
    try:
        buf.gen_corpus([0], [data_len])
        ch.plan([0], [data_len], data_len)
        ch.set_timing(True)
        for _ in range(3):
            ch.launch(buf.ptr)
        ms, n = ch.kernel_times()
        ch.set_timing(False)
        assert n == 3 and ms[0] > 0 and ms[2] > 0
        ch.set_timing(True, scan_only=True)          # the scan by the device clock (no events)
        for _ in range(2):
            ch.launch(buf.ptr)
        ms2, n2 = ch.kernel_times()
        ch.set_timing(False)
        assert n2 == 2 and ms2[0] > 0 and ms2[1] == ms2[2] == ms2[3] == 0
        ch.set_timing(True, scan_only=True, events=True)   # the scan by HIP events on its dispatch
        for _ in range(2):
            ch.launch(buf.ptr)
        ms3, n3 = ch.kernel_times()
        ch.set_timing(False)
        assert n3 == 2 and ms3[0] > 0 and ms3[1] == ms3[2] == ms3[3] == 0
        # the two measure the same kernel: the same order of magnitude (on a 64 MiB batch the
        # scan is ~20-40 us and its dispatch start-up is part of both)
        assert 0.5 * ms3[0] <= ms2[0] <= 2.0 * ms3[0], (ms2[0], ms3[0])
        # the raw modes keep their ABI-v2 meaning (2 = the scan by HIP events);
        # the device clock is mode 4; anything else is refused
        lib = syncr_amd.library()
        for mode, clock in ((2, False), (3, False), (4, True)):
            assert lib.syncr_cdc_set_timing(ch.handle, mode) == 0
            ch.launch(buf.ptr)
            m, k = ch.kernel_times()
            assert k == 1 and m[0] > 0 and m[1] == m[2] == 0, (mode, m, k)
        assert lib.syncr_cdc_set_timing(ch.handle, 5) == -22
        ch.set_timing(False)
        ch.fetch()
        st = ch.last_stats()
        assert st["tiles"] >= data_len // (144 * 128) and st["flags"] == 0
    finally:
        buf.free()


@pytest.mark.parametrize("flags", [syncr_amd.FLAG_RESOLVE_LANE, syncr_amd.FLAG_RESOLVE_NOBURST])
def test_resolve_variants_agree(kat_cases, flags):
    """Wave-per-file with burst (default), lane-per-file and wave without burst
    (params.flags, exact alternatives) give identical cuts on every KAT."""
    sel = [c for c in kat_cases if c["len"] <= 8 * M]
    alt = {}
    try:
        for c in sel:
            key = (c["chunk_bits"], c["max_chunk"], c["read_cap"])
            if key not in alt:
                alt[key] = syncr_amd.Chunker(*key, flags=flags)
            data = make_input(c["recipe"])
            assert ends_of(alt[key].cut_array(data)) == c["ends"], c["name"]
    finally:
        for ch in alt.values():
            ch.close()


def test_product_ignores_environment(kat_cases, monkeypatch):
    """the timing-only ablations and experimental kernels
    live only in the development library.  With every variable the round-1
    library read set to a non-exact or experimental value, the product still
    returns oracle-exact cuts and BLAKE3 hashes."""
    for k, v in {"SYNCR_CDC_ABLATE": "1", "SYNCR_B3_ABLATE": "1", "SYNCR_CDC_SCAN": "mfma",
                 "SYNCR_CDC_RUN": "48", "SYNCR_CDC_NB": "4", "SYNCR_CDC_NT": "0", "SYNCR_CDC_RESOLVE": "lane",
                 "SYNCR_B3_LOAD": "plain", "SYNCR_CDC_SCAN_GRID": "3", "SYNCR_CDC_SERIAL": "0"}.items():
        monkeypatch.setenv(k, v)
    with syncr_amd.Chunker() as ch:
        info = ch.info()
        assert info["run_bytes"] == 144 and info["scan_grid"] > 3
        data = O.xorshift_bytes(4242, 12 * M + 77)
        got = ch.chunk_bytes(data, hashed=True)
        ends = [c.offset + c.size for c in got]
        assert ends == O.chunk_production(data).tolist()
        for c in got:
            assert c.hash == O.blake3(data[c.offset:c.offset + c.size])
        for c in [k for k in kat_cases if k["len"] <= 4 * M][:12]:
            if (c["chunk_bits"], c["max_chunk"], c["read_cap"]) == (20, 16 * M, 2 * M):
                assert ends_of(ch.cut_array(make_input(c["recipe"]))) == c["ends"], c["name"]


def test_two_handles_interleaved_on_one_device():
    """Handles of one device order their scans (a scan waits for the other
    handle's last scan, cdc_api.cpp ScanOrder); interleaved launches on two
    handles and streams, each on its own copy of a corpus, stay exact."""
    lens = np.array([5 * M + 3, 0, 777, 3 * M, 40 * 1024] * 6, np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    span = int(lens.sum())
    hs = [syncr_amd.Chunker(), syncr_amd.Chunker()]
    bufs = []
    try:
        for k, h in enumerate(hs):
            b = syncr_amd.DeviceBuffer(h, span)
            b.gen_corpus(offs, lens, first_index=100 * k)
            h.plan(offs, lens, span)
            bufs.append(b)
        for step in range(12):
            h = hs[step % 2]
            h.launch(bufs[step % 2].ptr, hashed=(step % 3 == 0))
        for k, h in enumerate(hs):
            h.launch(bufs[k].ptr, hashed=True)
        for k, h in enumerate(hs):
            got = h.fetch(hashed=True)
            host = bufs[k].download(span)
            for i in range(lens.size):
                f = host[int(offs[i]): int(offs[i] + lens[i])]
                e = (got[i]["offset"] + got[i]["len"]).tolist()
                assert e == O.chunk_production(f).tolist(), (k, i)
                for c in got[i]:
                    o, n = int(c["offset"]), int(c["len"])
                    assert c["hash"].tobytes() == O.blake3(f[o:o + n])
    finally:
        for b in bufs:
            b.free()
        for h in hs:
            h.close()


def test_dedup_corpus_full_size():
    """SURVEY §8d config 5 at its full BASELINE size: 1000 variants of one 32 MiB
    random base, each with one 1-256 byte edit (50 % overwrite, 25 % insert,
    25 % delete) = ~32 GiB, device-resident, chunked AND hashed: every cut and
    every BLAKE3 bit-exact vs the oracle; boundary stability vs the base."""
    rng = np.random.default_rng(20251212)
    base = O.xorshift_bytes(31337, 32 * M)
    plan = []
    for _ in range(1000):
        pos = int(rng.integers(0, base.size))
        ln = int(rng.integers(1, 257))
        kind = ("overwrite", "overwrite", "insert", "delete")[int(rng.integers(0, 4))]
        ins = rng.integers(0, 256, ln, dtype=np.uint8)
        size = base.size + (ln if kind == "insert" else (-min(ln, base.size - pos) if kind == "delete" else 0))
        plan.append((kind, pos, ln, ins, size))
    lens = np.array([p[4] for p in plan], np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens)[:-1]
    total = int(lens.sum())
    buf = np.empty(total, np.uint8)
    edits = []
    for (kind, pos, ln, ins, size), o in zip(plan, offs.tolist()):
        f = buf[o:o + size]
        if kind == "overwrite":
            f[:] = base
            k = max(0, min(ln, base.size - pos))
            f[pos:pos + k] = ins[:k]
            edits.append((pos, 0))
        elif kind == "insert":
            f[:pos] = base[:pos]
            f[pos:pos + ln] = ins
            f[pos + ln:] = base[pos:]
            edits.append((pos, ln))
        else:
            d = min(ln, base.size - pos)
            f[:pos] = base[:pos]
            f[pos:] = base[pos + d:]
            edits.append((pos, -d))
    with syncr_amd.Chunker() as ch:
        dev = syncr_amd.DeviceBuffer(ch, total)
        try:
            dev.upload(buf)
            ch.plan(offs, lens, total)
            ch.launch(dev.ptr, hashed=True)
            got = ch.fetch(hashed=True)
        finally:
            dev.free()
    ref = O.chunk_batch(buf, offs, lens, nthreads=16)
    base_cuts = set(O.chunk_production(base).tolist())
    kept, starts, sizes = [], [], []
    for i in range(lens.size):
        e = ends_of(got[i])
        assert e == ref[i].tolist(), i
        starts.append(got[i]["offset"].astype(np.uint64) + offs[i])
        sizes.append(got[i]["len"].astype(np.uint64))
        pos, delta = edits[i]
        adj = {x - delta if x > pos else x for x in e}
        kept.append(len(adj & base_cuts) / len(base_cuts))
    want = O.blake3_batch(buf, np.concatenate(starts), np.concatenate(sizes), nthreads=16)
    assert np.array_equal(np.concatenate([g["hash"] for g in got]), want)
    assert np.median(kept) >= 0.9


def test_read_probe_reports_a_plausible_rate():
    """The streaming-read probe (bench.py's measured roofline denominator) runs
    over a resident buffer, writes nothing and reports best <= mean."""
    with syncr_amd.Chunker(device=0) as ch:
        n = 256 * M + 48                                  # ragged tail: not a multiple of a block step
        buf = syncr_amd.DeviceBuffer(ch, n)
        try:
            buf.gen_corpus(np.array([0], np.uint64), np.array([n], np.uint64))
            before = buf.download(4096)
            for nt in (True, False):
                best, mean = ch.read_probe(buf.ptr, n, reps=3, nt=nt)
                assert 0 < best <= mean
                assert 100.0 < n / (best / 1e3) / 1e9 < 20000.0          # GB/s
            assert np.array_equal(buf.download(4096), before)
            with pytest.raises(syncr_amd.SyncrCdcError):
                ch.read_probe(buf.ptr, 0, reps=1)
        finally:
            buf.free()


@pytest.mark.parametrize("bits,mx,cap", [(12, 16 << 20, 2 << 20), (16, 1 << 20, 70000), (14, 40000, 0),
                                         (10, 3000, 1000)])
def test_long_resolve_chains(chunkers, bits, mx, cap):
    """One 48 MiB file cut into thousands of chunks: the wave resolve walks
    hundreds of 64-candidate windows, its chained-hop bursts end on every
    kind of break (window end, read limit R, max-chunk cut, head hit), and
    the cuts a burst writes directly interleave with the gathered ones."""
    rng = np.random.default_rng(bits * 1000 + cap)
    data = rng.integers(0, 256, 48 * M, dtype=np.uint8)
    data[5 * M: 5 * M + 300000] = 7                       # a low-entropy stretch: max-chunk cuts
    ch = chunkers(bits, mx, cap)
    cuts = ch.cut_array(data)
    assert ends_of(cuts) == oracle_ends(data, bits, mx, cap)
    check_contiguous(cuts, data.size, mx)


def _split_corpus(bits, cap):
    from benchlib.workloads import periodic_pattern
    pat = periodic_pattern() if bits == 20 else None
    rng = np.random.default_rng(bits * 7919 + cap)
    files = []
    lo, hi = (34 * M, 44 * M) if bits == 10 else (5 * M, 14 * M)
    for k in range(3 if bits == 10 else 4):
        n = int(rng.integers(lo, hi))
        if pat is not None:                         # periodic with random glitches every ~1-3 MiB
            f = np.resize(pat, n)
            for g in rng.integers(0, n - 4096, 6).tolist():
                f[g: g + int(rng.integers(1, 3000))] = rng.integers(0, 256, 1, dtype=np.uint8)
        else:                                       # random: a candidate every ~2^bits bytes, many not cuts
            f = rng.integers(0, 256, n, dtype=np.uint8)
            f[n // 3: n // 3 + 200000] = 9          # a constant stretch: max-chunk cuts
        files.append(f)
    files.append(rng.integers(0, 256, 3 * M, dtype=np.uint8))       # below the split threshold
    lens = np.array([f.size for f in files], np.uint64)
    offs = np.zeros_like(lens)
    offs[1:] = np.cumsum(lens + 48)[:-1]
    span = int(offs[-1] + lens[-1]) + 16
    data = np.zeros(span, np.uint8)
    for o, f in zip(offs.tolist(), files):
        data[o:o + f.size] = f
    return data, offs, lens


def _split_oracle(data, offs, lens, bits, mx, cap):
    return [(O.chunk_production_window(data[o:o + n], bits, mx, cap) if cap else
             O.chunk_ideal(data[o:o + n], bits, mx)).tolist() for o, n in zip(offs.tolist(), lens.tolist())]


@pytest.mark.parametrize("bits,mx,cap", [(8, 4096, 3000), (8, 1 << 16, 0), (10, 1 << 14, 2 << 20),
                                         (20, 16 << 20, 2 << 20), (20, 16 << 20, 0)])
def test_split_walks(bits, mx, cap):
    """Split walks of long files: files of >= SPLIT_MIN_BYTES
    (256 KiB) holding >= 2 x SPLIT_SEGC (8192) candidates are walked in
    segments of 8192 candidates by extra resolve waves and stitched where a
    walk lands on a segment's start with its start state; the handle launches
    the extra waves once a fetch has seen >= 64 Ki candidates at >= 1 per
    16 KiB.  Mixed content makes segment starts that are not cuts, read-limit
    mismatches and aborted segment walks; every file must equal the oracle and
    the unsplit walk (SYNCR_CDC_FLAG_RESOLVE_NOSPLIT), and the split run must
    have split files and adopted segment walks (syncr_cdc_split_stats)."""
    data, offs, lens = _split_corpus(bits, cap)
    got, stats = {}, {}
    for flags in (0, syncr_amd.FLAG_RESOLVE_NOSPLIT):
        with syncr_amd.Chunker(bits, mx, cap, flags=flags) as ch:
            # the first call's fetch turns the split hint on: the second call
            # (and the re-runs of the first) walk split
            got[flags] = [ends_of(r) for r in ch.batch_arrays(data, offs, lens)]
            got[flags + 100] = [ends_of(r) for r in ch.batch_arrays(data, offs, lens)]
            stats[flags] = ch.split_stats()
    want = _split_oracle(data, offs, lens, bits, mx, cap)
    for i in range(lens.size):
        for k in got:
            assert got[k][i] == want[i], (i, int(lens[i]), bits, mx, cap, k)
    sp = stats[0]
    assert sp["workers"] > 0 and sp["files_split"] >= 1 and sp["segments"] >= 1, sp
    assert sp["walked"] >= 1 and sp["adopted"] >= 1 and sp["giveups"] == 0, sp
    assert stats[syncr_amd.FLAG_RESOLVE_NOSPLIT]["workers"] == 0


@pytest.mark.parametrize("bits,mx,cap", [(8, 4096, 3000), (20, 16 << 20, 2 << 20)])
def test_split_workers_give_up(bits, mx, cap):
    """a split worker's waits are bounded; one that gives up
    leaves its segments to the file walkers, which never wait.  With
    SYNCR_CDC_FLAG_SPLIT_NOWAIT every worker gives up at once: no segment walk
    is done or adopted, and every file is still oracle-exact."""
    data, offs, lens = _split_corpus(bits, cap)
    with syncr_amd.Chunker(bits, mx, cap, flags=syncr_amd.FLAG_SPLIT_NOWAIT) as ch:
        ch.batch_arrays(data, offs, lens)
        got = [ends_of(r) for r in ch.batch_arrays(data, offs, lens)]
        sp = ch.split_stats()
    assert got == _split_oracle(data, offs, lens, bits, mx, cap)
    assert sp["workers"] > 0 and sp["files_split"] >= 1, sp
    assert sp["giveups"] == sp["workers"] and sp["walked"] == 0 and sp["adopted"] == 0, sp


def test_fetch_reruns_reported():
    """syncr_cdc_fetch_reruns: a first launch whose capacities are too small
    (periodic data: a candidate every 64 bytes) is re-run inside the fetch and
    says so; the next launch, with the grown capacities, needs none.  bench.py
    re-times its region when its first fetch reports a re-run."""
    import bench
    data = np.resize(bench.periodic_pattern(), 6 * M + 5)
    with syncr_amd.Chunker(20, 16 << 20, 2 << 20) as ch:
        buf = syncr_amd.DeviceBuffer(ch, data.size)
        try:
            buf.upload(data)
            offs = np.array([0], np.uint64)
            lens = np.array([data.size], np.uint64)
            ch.plan(offs, lens, data.size)
            ch.launch(buf.ptr)
            first = ch.fetch()
            assert ch.fetch_reruns() > 0
            ch.fetch()                                   # a second fetch of the same launch: still counted
            assert ch.fetch_reruns() > 0
            ch.launch(buf.ptr)
            again = ch.fetch()
            assert ch.fetch_reruns() == 0
            assert ends_of(first[0]) == ends_of(again[0]) == O.chunk_production_window(data).tolist()
        finally:
            buf.free()


def test_launches_on_alternating_streams():
    """One handle launched on two caller streams in turn with no fetch in
    between (include/syncr_cdc.h: a launch on another stream waits for the
    previous launch's stream), over a periodic + constant + random batch whose
    first fetch must re-run the launch (dense tiles not yet seen, grown
    capacities).  Cuts and chunk hashes against the oracle."""
    from benchlib import legs as LG
    from benchlib import workloads as WL
    files = LG.dense_subset_files()[:6] + [O.xorshift_bytes(4321, 9 * M + 11)]
    lens = np.array([f.size for f in files], np.uint64)
    offs = WL.offsets_of(lens)
    buf_h = np.concatenate(files)
    want = [O.chunk_production_window(f).tolist() for f in files]
    with syncr_amd.Chunker() as ch, syncr_amd.Chunker() as a1, syncr_amd.Chunker() as a2:
        streams = (a1.stream, a2.stream)
        assert streams[0] and streams[1] and streams[0] != streams[1]
        d = syncr_amd.DeviceBuffer(ch, buf_h.size)
        try:
            d.upload(buf_h)
            ch.plan(offs, lens, buf_h.size)
            for rnd in range(2):
                for k in range(7):
                    ch.launch(d.ptr, stream=streams[k % 2], hashed=(k % 3 == 0))
                got = ch.fetch(hashed=True)           # the last launch (k = 6) was hashed
                if rnd == 0:
                    assert ch.fetch_reruns() > 0      # the re-run happened inside fetch
                for g, w, f in zip(got, want, files):
                    assert ends_of(g) == w
                    if g.size:
                        h = O.blake3_batch(f, g["offset"].astype(np.uint64), g["len"].astype(np.uint64), nthreads=8)
                        assert np.array_equal(g["hash"], h)
                # the handle's own stream after the caller's
                ch.launch(d.ptr)
                assert all(ends_of(g) == w for g, w in zip(ch.fetch(), want))
        finally:
            d.free()


def test_handles_in_flight_together():
    """Scans of different handles on one device are not ordered (a second
    handle's scan takes the CUs as the first one's last work units end).  Three
    handles with different batches -- small random files (the CU schedule), a
    periodic + constant + random batch (dense tiles, a re-run inside fetch) and
    one larger random batch (stream tiles) -- launched on their own streams three
    times over with no wait in between; every cut and chunk hash against the
    oracle."""
    from benchlib import legs as LG
    small = [O.xorshift_bytes(60 + k, 300_000 + 77 * k) for k in range(12)]
    dense = LG.dense_subset_files()[:4] + [O.xorshift_bytes(4323, 5 * M + 3)]
    big = [O.xorshift_bytes(71 + k, 24 * M + 1000 * k) for k in range(3)]
    batches = [small, dense, big]
    hs, bufs = [], []
    try:
        for files in batches:
            lens = np.array([f.size for f in files], np.uint64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
            h = syncr_amd.Chunker()
            b = syncr_amd.DeviceBuffer(h, int(lens.sum()))
            b.upload(np.concatenate(files))
            h.plan(offs, lens, int(lens.sum()))
            hs.append(h)
            bufs.append(b)
        for rnd in range(3):
            for h, b in zip(hs, bufs):
                h.launch(b.ptr, hashed=True)
        for h, files in zip(hs, batches):
            got = h.fetch(hashed=True)
            for g, f in zip(got, files):
                assert ends_of(g) == O.chunk_production_window(f).tolist()
                if g.size:
                    want = O.blake3_batch(f, g["offset"].astype(np.uint64), g["len"].astype(np.uint64), nthreads=8)
                    assert np.array_equal(g["hash"], want)
    finally:
        for b in bufs:
            b.free()
        for h in hs:
            h.close()


def test_plans_on_caller_stream_reuse_staging():
    """plan leaves its table upload in flight on the handle's stream; a launch on
    a caller stream waits for it, and the next plan reuses the pinned staging
    only once that upload completed.  Twenty plans of different file tables
    (one plan replaced before any launch), each launched on a caller stream and
    fetched with hashes, against the oracle."""
    rng = np.random.default_rng(77)
    files = [O.xorshift_bytes(900 + k, int(n)) for k, n in enumerate(rng.integers(0, 3 * M, 24))]
    with syncr_amd.Chunker() as ch, syncr_amd.Chunker() as other:
        for r in range(20):
            pick = [files[(r + 3 * j) % len(files)] for j in range(1 + r % 5)]
            lens = np.array([f.size for f in pick], np.uint64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
            host = np.concatenate(pick) if lens.sum() else np.zeros(1, np.uint8)
            d = syncr_amd.DeviceBuffer(ch, max(host.size, 1))
            try:
                d.upload(host)
                if r == 7:                                   # a plan replaced before its launch
                    ch.plan(offs[:1], lens[:1], int(lens.sum()))
                ch.plan(offs, lens, int(lens.sum()))
                ch.launch(d.ptr, stream=other.stream, hashed=True)
                got = ch.fetch(hashed=True)
            finally:
                d.free()
            for g, f in zip(got, pick):
                assert ends_of(g) == O.chunk_production_window(f).tolist()
                if g.size:
                    h = O.blake3_batch(f, g["offset"].astype(np.uint64), g["len"].astype(np.uint64), nthreads=8)
                    assert np.array_equal(g["hash"], h)


def test_small_batches_back_to_back_stable():
    """Small batches run the CU scan schedule (a workgroup per CU, a ring of
    group ids in LDS).  LDS survives between workgroups: a ring slot left by an
    earlier launch on the same CU once carried the tag a wave was waiting for,
    and the wave scanned a stale group (lost and doubled tiles: 2 of 10 000
    files wrong in the bench's ingest leg).  Two handles with batches of
    different sizes (last rows of their groups mostly past the batch end)
    launch back to back, 12 times each; every launch equals the oracle."""
    sizes = [(211, (1 << 20) + 4093), (97, (1 << 20) - 777)]
    hs, bufs, refs, plans = [], [], [], []
    try:
        for nfiles, flen in sizes:
            ch = syncr_amd.Chunker(chunk_bits=20, max_chunk=16 << 20, read_cap=2 << 20)
            hs.append(ch)
            lens = np.full(nfiles, flen, np.uint64)
            offs = np.arange(nfiles, dtype=np.uint64) * np.uint64(flen)
            span = int(lens.sum())
            buf = syncr_amd.DeviceBuffer(ch, span)
            bufs.append(buf)
            buf.gen_corpus(offs, lens, indices=np.arange(nfiles, dtype=np.uint64) + 7 * nfiles)
            ch.plan(offs, lens, span)
            host = buf.download(span)
            refs.append([r.tolist() for r in O.chunk_batch(host, offs, lens, read_cap=2 << 20,
                                                           mode=O.MODE_PRODUCTION)])
            plans.append(nfiles)
            del host
        for it in range(12):
            for k, ch in enumerate(hs):
                ch.launch(bufs[k].ptr)
            for k, ch in enumerate(hs):
                res = ch.fetch()
                bad = [i for i in range(plans[k]) if ends_of(res[i]) != refs[k][i]]
                assert not bad, (it, k, bad[:5])
    finally:
        for b in bufs:
            b.free()
        for ch in hs:
            ch.close()


# cdc_kernels.hip SCAN_ST_MIN_TILES_PER_WAVE / SCAN_DYN_MIN_TILES_PER_WAVE: the tests pin the
# library's choice at these thresholds through syncr_cdc_last_scan (the host never restates it)
SCAN_ST_MIN_TILES_PER_WAVE = 24
SCAN_DYN_MIN_TILES_PER_WAVE = 96

@pytest.mark.parametrize("per_wave,below", [(SCAN_ST_MIN_TILES_PER_WAVE, False), (SCAN_ST_MIN_TILES_PER_WAVE, True)])
def test_stream_tile_threshold_edge_vs_oracle(per_wave, below):
    """The scans either side of the library's thresholds (cdc_kernels.hip
    launch_scan / st_segs), as syncr_cdc_last_scan reports them: a batch of
    exactly grid x 24 tiles whose last tile holds one byte (stream tiles of
    9-segment streams; the batch's last stream tile is mostly past the span: the
    clamped DMA path) and one tile less (the CU schedule).  Random files with periodic-64 and constant ones at
    chunk_bits 13: every file's cuts vs the oracle."""
    from benchlib.workloads import periodic_pattern
    bits, cap = 13, 256 << 10
    rng = np.random.default_rng(24 + below)
    ch = syncr_amd.Chunker(chunk_bits=bits, max_chunk=16 << 20, read_cap=cap)
    try:
        info = ch.info()
        tb = info["tile_bytes"]
        ntiles = info["scan_grid"] * per_wave
        span = (ntiles - 1) * tb + (0 if below else 1)
        lens = []
        while sum(lens) < span:
            lens.append(int(rng.integers(1, 24 << 20)))
        lens[-1] -= sum(lens) - span
        if lens[-1] == 0:
            lens.pop()
        lens = np.array(lens, np.uint64)
        offs = np.zeros_like(lens)
        offs[1:] = np.cumsum(lens)[:-1]
        assert int(lens.sum()) == span
        want, kind, segs = (("cdc_scan_kernel", "cu_schedule", 0) if below else
                            ("cdc_scan_st_kernel", "stream_tiles", 9))
        buf = syncr_amd.DeviceBuffer(ch, span)
        try:
            buf.gen_corpus(offs, lens, indices=np.arange(lens.size, dtype=np.uint64) + 7001)
            pat = periodic_pattern()
            for i in range(lens.size):
                if i % 5 == 2:
                    buf.upload(np.resize(pat, int(lens[i])), offset=int(offs[i]))
                elif i % 5 == 4:
                    buf.upload(np.full(int(lens[i]), 0xA5, np.uint8), offset=int(offs[i]))
            ch.plan(offs, lens, span)
            ch.launch(buf.ptr)
            res = ch.fetch()
            rep = ch.last_scan()                   # the library's own report (syncr_cdc_last_scan)
            assert rep["kernel"] == want and rep["kind"] == kind and rep["st_segments"] == segs, rep
            assert rep["tiles"] == ntiles - below and rep["waves"] == info["scan_grid"], rep
            host = buf.download(span)
            print(f"{want} edge batch: {lens.size} files, {span} bytes; oracle next", flush=True)
        finally:
            buf.free()
        ref = O.chunk_batch(host, offs, lens, bits=bits, read_cap=cap, mode=O.MODE_PRODUCTION_WINDOW)
        bad = [i for i in range(lens.size) if ends_of(res[i]) != ref[i].tolist()]
        assert not bad, bad[:10]
    finally:
        ch.close()


@pytest.mark.parametrize("bits,cap", [(12, 64 << 10), (20, 2 << 20)])
def test_large_batch_stream_tiles_vs_oracle(bits, cap):
    """A batch well inside the stream-tile scan's range (96 tiles per scan wave;
    the product's scan from 24) with random, periodic-64 and constant
    files of ragged sizes, at a small mask (dirty groups in most segments: slot
    overflow and dense marks) and at the production mask: every file's cuts vs
    the oracle."""
    from benchlib.workloads import periodic_pattern
    rng = np.random.default_rng(bits * 7919 + cap)
    ch = syncr_amd.Chunker(chunk_bits=bits, max_chunk=16 << 20, read_cap=cap)
    try:
        info = ch.info()
        need = info["scan_grid"] * 96 * info["tile_bytes"] + (1 << 20)      # well inside the stream-tile range
        lens = []
        while sum(lens) < need:
            lens.append(int(rng.integers(1, 96 << 20)))
        lens = np.array(lens, np.uint64)
        offs = np.zeros_like(lens)
        offs[1:] = np.cumsum(lens)[:-1]
        span = int(lens.sum())
        buf = syncr_amd.DeviceBuffer(ch, span)
        try:
            buf.gen_corpus(offs, lens, indices=np.arange(lens.size, dtype=np.uint64) + 100003)
            pat = periodic_pattern()
            for i in range(lens.size):
                if i % 8 == 3:                     # periodic-64 file
                    buf.upload(np.resize(pat, int(lens[i])), offset=int(offs[i]))
                elif i % 8 == 6:                   # one constant byte
                    buf.upload(np.full(int(lens[i]), 0x5A, np.uint8), offset=int(offs[i]))
            ch.plan(offs, lens, span)
            ch.launch(buf.ptr)
            res = ch.fetch()
            assert ch.last_scan()["kind"] == "stream_tiles" and ch.last_scan()["st_segments"] == 9, ch.last_scan()
            host = buf.download(span)
            print(f"stream-tile batch: {lens.size} files, {span / 2**30:.2f} GiB chunked; oracle next", flush=True)
        finally:
            buf.free()
        # the windowed restatement of the production loop: the literal loop memmoves its
        # 16 MiB buffer after every 64-byte chunk of a periodic file (quadratic)
        ref = O.chunk_batch(host, offs, lens, bits=bits, read_cap=cap, mode=O.MODE_PRODUCTION_WINDOW)
        bad = [i for i in range(lens.size) if ends_of(res[i]) != ref[i].tolist()]
        assert not bad, bad[:10]
    finally:
        ch.close()


def test_dense_heavy_handle_large_batch_dynamic_tiles_vs_oracle():
    """after a batch with >= 1 % dense tiles a handle scans its
    next large batches (>= 96 tiles per wave) by tiles with dynamic groups.  A
    batch whose tile count leaves a partial last round (ntiles % (8 x grid) in
    [1, 2 x grid)) makes groups that end at their first tile; a lost grab there
    used to drop a group (its candidates vanished without an error).  One
    handle: a dense-heavy batch first, then such a batch of random, periodic-64
    and constant files; the library must report the tile scan, and every file's
    cuts must equal the oracle's."""
    from benchlib.workloads import periodic_pattern
    bits, cap = 20, 2 << 20
    rng = np.random.default_rng(96)
    ch = syncr_amd.Chunker(chunk_bits=bits, max_chunk=16 << 20, read_cap=cap)
    try:
        info = ch.info()
        tb, grid = info["tile_bytes"], info["scan_grid"]
        pat = periodic_pattern()
        # 1: a dense-heavy batch (periodic data: every tile dense)
        dense = np.resize(pat, 64 << 20)
        first = ch.batch_arrays(dense, [0], [dense.size])[0]
        assert ends_of(first) == O.chunk_production_window(dense).tolist()
        assert ch.last_stats()["dense_tiles"] * 100 >= -(-dense.size // tb)
        # 2: the large batch, a partial last round of single-tile groups
        rounds = -(-grid * SCAN_DYN_MIN_TILES_PER_WAVE // (8 * grid))
        ntiles = rounds * 8 * grid + grid // 2 + 3
        span = (ntiles - 1) * tb + 777
        lens = []
        while sum(lens) < span:
            lens.append(int(rng.integers(1, 64 << 20)))
        lens[-1] -= sum(lens) - span
        if lens[-1] == 0:
            lens.pop()
        lens = np.array(lens, np.uint64)
        offs = np.zeros_like(lens)
        offs[1:] = np.cumsum(lens)[:-1]
        buf = syncr_amd.DeviceBuffer(ch, span)
        try:
            buf.gen_corpus(offs, lens, indices=np.arange(lens.size, dtype=np.uint64) + 960001)
            for i in range(lens.size):
                if i % 16 == 5:
                    buf.upload(np.resize(pat, int(lens[i])), offset=int(offs[i]))
                elif i % 16 == 11:
                    buf.upload(np.full(int(lens[i]), 0x3C, np.uint8), offset=int(offs[i]))
            ch.plan(offs, lens, span)
            ch.launch(buf.ptr)
            rep = ch.last_scan()
            assert rep["kind"] == "tiles_dynamic" and rep["kernel"] == "cdc_scan_kernel", rep
            assert rep["tiles"] == ntiles and ntiles % (8 * grid) in range(1, 2 * grid), rep
            res = ch.fetch()
            host = buf.download(span)
            print(f"dynamic-tile batch: {lens.size} files, {span / 2**30:.2f} GiB; oracle next", flush=True)
        finally:
            buf.free()
        ref = O.chunk_batch(host, offs, lens, bits=bits, read_cap=cap, mode=O.MODE_PRODUCTION_WINDOW)
        bad = [i for i in range(lens.size) if ends_of(res[i]) != ref[i].tolist()]
        assert not bad, bad[:10]
    finally:
        ch.close()


def test_stream_destroyed_after_fetch():
    """the header lets a caller destroy its stream once the launch on
    it has been fetched.  Launch on a caller stream (another handle's, destroyed
    with that handle), fetch, destroy it, then plan, launch on the handle's own
    stream and fetch again: nothing may touch the destroyed stream, and the cuts
    stay exact."""
    data = O.xorshift_bytes(515, 9 * M + 3)
    want = O.chunk_production(data).tolist()
    with syncr_amd.Chunker() as ch:
        buf = syncr_amd.DeviceBuffer(ch, data.size)
        try:
            buf.upload(data)
            for rep in range(3):
                other = syncr_amd.Chunker()
                ch.plan([0], [data.size], data.size)
                ch.launch(buf.ptr, stream=other.stream)
                assert ends_of(ch.fetch()[0]) == want
                other.close()                           # destroys the stream the launch ran on
                ch.plan([0], [data.size], data.size)
                ch.launch(buf.ptr)
                assert ends_of(ch.fetch()[0]) == want
                ch.synchronize()
        finally:
            buf.free()
