"""Full-size parity of the HIP engine against the golden per-file digests of
the CPU oracle (tests/golden/*_digests.npz, made by
tests/golden/make_corpus_digests.py): every file of the zipf10k corpus (SURVEY
§8d config 3) in both semantics and with chunk hashes, the device-built dedup
corpus (config 5) and the adversarial dense workload -- the same checks
bench.py's parity leg reports on the driver's box.  Bar: bit-exact."""
import numpy as np
import pytest

import syncr_amd
from benchlib import golden as G
from benchlib import legs as L
from benchlib import workloads as WL

pytestmark = pytest.mark.gpu
M = 1 << 20


def test_zipf10k_every_file_vs_golden_digests():
    lens = WL.zipf_sizes()
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    idx = np.arange(lens.size)
    with syncr_amd.Chunker() as ch:
        buf = syncr_amd.DeviceBuffer(ch, span)
        try:
            buf.gen_corpus(offs, lens)
            ch.plan(offs, lens, span)
            ch.launch(buf.ptr, hashed=True)
            p = G.check_files("zipf10k", ch.fetch(hashed=True), idx, hashed=True)
            assert p["files"] == 10000 and p["mismatches"] == 0, p
            ideal = L.ideal_leg(buf, offs, lens, idx, 0)
            assert ideal["files"] == 10000 and ideal["mismatches"] == 0, ideal
        finally:
            buf.free()


def test_dedup_built_on_device_vs_golden_digests():
    """The dedup corpus assembled in HBM (gen_corpus + syncr_cdc_memcpy_d2d)
    equals the host-built variants the golden digests were computed from."""
    r = L.dedup_leg(0, steps=2, warmup=1)
    assert r["parity"]["files"] == 1000 and r["parity"]["mismatches"] == 0, r["parity"]
    assert r["parity_hashed"]["mismatches"] == 0, r["parity_hashed"]
    assert r["stability"]["kept_median"] >= 0.9


def test_dense_workload_vs_golden_digests():
    r = L.dense_leg(0, steps=2, warmup=1)
    assert r["parity"]["files"] == 10000 and r["parity"]["mismatches"] == 0, r["parity"]
    assert r["parity_hashed"]["mismatches"] == 0, r["parity_hashed"]
    assert r["dense_tiles"] > 0 and r["split"]["adopted"] > 0, r


def test_parity_legs_of_smoke_and_bench():
    for leg in (L.kat_leg, L.blake3_vectors_leg, L.dense_subset_leg):
        r = leg(0)
        assert r["mismatches"] == 0 and r.get("hash_mismatches", 0) == 0, (leg.__name__, r)
    r = L.ingest_multi_leg(0)
    assert r["parity"]["mismatches"] == 0 and r["parity"]["files"] > 500, r


def test_memcpy_d2d():
    with syncr_amd.Chunker() as ch:
        a = syncr_amd.DeviceBuffer(ch, 1 << 20)
        b = syncr_amd.DeviceBuffer(ch, 1 << 20)
        try:
            a.gen_corpus([0], [1 << 20])
            b.upload(np.zeros(1 << 20, np.uint8))
            b.copy_from(a.ptr + 5, 1000, offset=77)
            ch.synchronize()
            ha, hb = a.download(), b.download()
            assert np.array_equal(hb[77:1077], ha[5:1005]) and not hb[:77].any() and not hb[1077:].any()
        finally:
            a.free()
            b.free()


@pytest.mark.parametrize("nshards", [2, 8])
def test_strong_shards_vs_golden(nshards):
    """BASELINE config 4's per-rank batches (bench.py --gpus N --scaling strong:
    zipf10k LPT-sharded per file, benchlib/workloads.py lpt_shard) through the
    product path, one shard at a time on this GPU: every file of every shard,
    cuts and chunk hashes, against the golden digests; the shards together are
    exactly the 10 000 files (file_operations.rs:599-605,721-788: files are
    independent, so sharding cannot change a file's chunks)."""
    sizes = WL.zipf_sizes()
    shards = WL.lpt_shard(sizes, nshards)
    assert np.array_equal(np.sort(np.concatenate(shards)), np.arange(sizes.size))
    biggest = max(int(sizes[s].sum()) for s in shards)
    files = 0
    with syncr_amd.Chunker() as ch:
        buf = syncr_amd.DeviceBuffer(ch, biggest)
        try:
            for sh in shards:
                lens = sizes[sh]
                offs = WL.offsets_of(lens)
                buf.gen_corpus(offs, lens, indices=sh.astype(np.uint64))
                ch.plan(offs, lens, int(lens.sum()))
                ch.launch(buf.ptr, hashed=True)
                p = G.check_files("zipf10k", ch.fetch(hashed=True), sh, hashed=True)
                assert p["files"] == sh.size and p["mismatches"] == 0, p
                files += p["files"]
        finally:
            buf.free()
    assert files == sizes.size


def test_stream_tiles_back_to_back_launches_vs_golden():
    """The stream-tile scan's asynchronous ST grab (cdc_kernels.hip grab_async:
    an asm atomic whose result is read a segment later) across back-to-back
    launches of one plan with no fetch between them (the bench's timed steps),
    then a fetch: config 4's N = 8 rank-0 batch (35 tiles per scan wave, stream
    tiles; the library's own report says so), every file's cuts and hashes
    against the golden digests, twice."""
    sizes = WL.zipf_sizes()
    sh = WL.lpt_shard(sizes, 8)[0]
    lens = sizes[sh]
    offs = WL.offsets_of(lens)
    with syncr_amd.Chunker() as ch:
        buf = syncr_amd.DeviceBuffer(ch, int(lens.sum()))
        try:
            buf.gen_corpus(offs, lens, indices=sh.astype(np.uint64))
            ch.plan(offs, lens, int(lens.sum()))
            for rep in range(2):
                for _ in range(4):
                    ch.launch(buf.ptr, hashed=True)
                got = ch.fetch(hashed=True)
                assert ch.last_scan()["kind"] == "stream_tiles", ch.last_scan()
                p = G.check_files("zipf10k", got, sh, hashed=True)
                assert p["files"] == sh.size and p["mismatches"] == 0, (rep, p)
        finally:
            buf.free()


def test_shard_leg_reports_every_shard():
    r = L.shard_leg(0, steps=2, warmup=1, nshards=8)
    assert len(r["shards"]) == 8 and r["parity"]["files"] == 10000 and r["parity"]["mismatches"] == 0, r
    assert r["projected_value"] > 0 and all(s["scan_frac"] for s in r["shards"])
