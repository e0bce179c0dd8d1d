"""CPU oracle (oracle/bup_oracle.c) pinned against the golden fixtures and the
structural tests of the reference (tests/chunking_test.rs,
tests/protocol_list_test.rs:305-400).  No GPU needed."""
import numpy as np
import pytest

from golden_inputs import make_input
from oracle import oracle as O

M = 1 << 20


def _ideal_or_prod(data, c):
    if c["read_cap"]:
        return O.chunk_production(data, c["chunk_bits"], c["max_chunk"], c["read_cap"])
    return O.chunk_ideal(data, c["chunk_bits"], c["max_chunk"])


def test_golden_cases_literal(kat_cases):
    for c in kat_cases:
        data = make_input(c["recipe"])
        assert data.size == c["len"]
        ends = _ideal_or_prod(data, c)
        assert ends.tolist() == c["ends"], c["name"]


def test_golden_cases_closed_form(kat_cases):
    for c in kat_cases:
        if c["len"] > 8 * M:
            continue
        data = make_input(c["recipe"])
        ends = O.chunk_closed_form(data, c["chunk_bits"], c["max_chunk"], c["read_cap"])
        assert ends.tolist() == c["ends"], c["name"]


def test_survey_appendix_a_values(kat_cases):
    by = {c["name"]: c for c in kat_cases}
    first = [(0, 1001954), (1001954, 132287), (1134241, 745223), (1879464, 867950),
             (2747414, 349596), (3097010, 994949)]
    for tag in ("prod", "ideal"):
        c = by[f"xorshift64M_{tag}"]
        assert c["n_chunks"] == 81
        assert O.ends_to_cuts(c["ends"])[:6] == first
    assert by["xorshift64M_zero3M_ideal"]["n_chunks"] == 76
    assert O.ends_to_cuts(by["xorshift64M_zero3M_ideal"]["ends"])[:3] == [
        (0, 4091959), (4091959, 2597299), (6689258, 166127)]
    assert by["xorshift64M_zero3M_prod"]["n_chunks"] == 78
    assert O.ends_to_cuts(by["xorshift64M_zero3M_prod"]["ends"])[:5] == [
        (0, 2097152), (2097152, 1994807), (4091959, 2199497), (6291456, 397802), (6689258, 166127)]
    assert by["const_A_50M_ideal"]["n_chunks"] == 4
    assert by["const_A_50M_prod"]["n_chunks"] == 25
    assert by["xorshift256M_ideal"]["n_chunks"] == 328
    assert by["small_prod"]["ends"] == [5]
    assert by["empty_prod"]["ends"] == []


def test_formulations_agree_random():
    rng = np.random.default_rng(1)
    for trial in range(40):
        n = int(rng.integers(0, 200_000))
        bits = int(rng.integers(6, 18))
        mx = int(rng.integers(1, 1 << (bits + 3)))
        cap = int(rng.choice([0, 1, 63, 64, 65, 1000, 1 << 16]))
        data = rng.integers(0, 256, n, dtype=np.uint8)
        if trial % 4 == 0:
            data = (data & 3).astype(np.uint8)           # low entropy
        lit = O.chunk_production(data, bits, mx, cap) if cap else O.chunk_ideal(data, bits, mx)
        assert np.array_equal(lit, O.chunk_closed_form(data, bits, mx, cap)), (trial, n, bits, mx, cap)


def test_window_locality():
    """rollsum/bup selftest style: the digest only depends on
    the last 64 bytes."""
    buf = O.xorshift_bytes(12345, 4096)
    for n in (65, 100, 4096):
        assert O.digest_after(buf[:n]) == O.digest_after(buf[1:n])
    assert O.digest_after(buf[:67]) == O.digest_after(buf[3:67])


def test_constant_bytes_never_hit():
    for v in range(256):
        d = np.full(5000, v, np.uint8)
        for bits in (13, 20):
            assert O.chunk_ideal(d, bits, 1 << 30).tolist() == [5000]


def test_chunking_test_rs_structural():
    """tests/chunking_test.rs assertions, on the oracle (bits 13, MAX 128 KiB)."""
    from golden_inputs import _chunking_test_input as inp
    mx = (1 << 13) * 16
    cut = lambda d: O.ends_to_cuts(O.chunk_ideal(np.frombuffer(d, np.uint8), 13, mx))
    assert cut(inp("deterministic")) == cut(inp("deterministic"))               # :11-23
    assert cut(inp("small_file")) == [(0, 10)]                                  # :26-34
    assert cut(inp("empty_file")) == []                                         # :37-43
    for nm in ("large_file", "binary_data", "identical_blocks", "from_file", "offset_progression"):
        cs = cut(inp(nm))                                                       # :46-73,110-167
        assert cs and sum(s for _, s in cs) == len(inp(nm))
        assert all(o == sum(s for _, s in cs[:i]) for i, (o, _) in enumerate(cs))
    assert all(s <= mx for _, s in cut(inp("boundaries")))                      # :95-108
    assert len(cut(inp("content_shifting_2"))) >= len(cut(inp("content_shifting_1")))  # :76-92


def test_protocol_list_pins():
    """tests/protocol_list_test.rs:305-400 pins on production semantics."""
    assert O.ends_to_cuts(O.chunk_production(b"small")) == [(0, 5)]
    big = np.full(50 * M, ord("A"), np.uint8)
    e = O.chunk_production(big)
    assert len(e) > 1 and int(e[-1]) == big.size
    x = np.full(100000, ord("X"), np.uint8)
    cs = O.ends_to_cuts(O.chunk_production(x))
    assert cs[0][0] == 0 and sum(s for _, s in cs) == 100000


def test_uniform_corpus_fixture(uniform_corpus_golden):
    g = uniform_corpus_golden
    lens = np.full(g["files"], g["file_len"], np.uint64)
    buf, offs = O.corpus_fill(lens)
    ends = O.chunk_batch(buf, offs, lens)
    assert [e.tolist() for e in ends] == g["ends"]


def test_corpus_seed_rule():
    # file i = xorshift64 seeded 0x9E3779B97F4A7C15*(i+1), 64 outputs discarded
    buf, offs = O.corpus_fill(np.array([100, 7, 0, 33], np.uint64), first_index=5)
    for j, (o, n) in enumerate(zip(offs.tolist(), [100, 7, 0, 33])):
        ref = O.xorshift_bytes((0x9E3779B97F4A7C15 * (5 + j + 1)) % 2**64, n, discard=64)
        assert np.array_equal(buf[o:o + n], ref)


def test_window_variant_equals_literal_loop():
    """orc_chunk_production_window (no copy_within) == the literal loop, on
    random, low-entropy, periodic (a cut every 64 bytes) and zero data, with and
    without the read cap -- it stands in for the literal loop only where the
    literal loop's O(buffer) memmove per chunk would take hours."""
    import bench
    pat = bench.periodic_pattern()
    inputs = [O.xorshift_bytes(31, 5 * M + 3), np.resize(pat, 300 * 1024 + 7),
              (O.xorshift_bytes(32, 3 * M) & 3).astype(np.uint8), np.zeros(5 * M + 1, np.uint8),
              np.concatenate([np.resize(pat, M), O.xorshift_bytes(33, 2 * M)])]
    for data in inputs:
        for bits, mx, cap in ((20, 16 * M, 2 * M), (20, 16 * M, 0), (13, 1 << 17, 3000), (8, 4096, 1000)):
            assert np.array_equal(O.chunk_production_window(data, bits, mx, cap),
                                  O.chunk_production(data, bits, mx, cap)), (data.size, bits, mx, cap)
    assert O.chunk_production_window(np.zeros(0, np.uint8)).size == 0
