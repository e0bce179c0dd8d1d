"""Randomized GPU parity (hypothesis, derandomized so every run draws the same
cases): batches of files of random sizes, gaps and contents, at random chunk
parameters, chunked AND hashed on the GPU, bit-exact against the oracle's
compute_file_chunks / chunk_data loops (file_operations.rs:721-788,
tests/chunking_test.rs:170-192) and its BLAKE3 (util.rs:57-59)."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import oracle as O

pytestmark = pytest.mark.gpu

PARAMS = [(1, 4096, 0), (5, 1000, 333), (8, 4096, 3000), (13, 128 * 1024, 0), (13, 128 * 1024, 64 * 1024),
          (16, 1 << 20, 70000), (20, 16 << 20, 2 << 20), (24, 300000, 0)]


@st.composite
def batches(draw):
    params = draw(st.sampled_from(PARAMS))
    nf = draw(st.integers(0, 12))
    sizes = draw(st.lists(st.one_of(st.integers(0, 70), st.integers(0, 5000), st.integers(0, 400000)),
                          min_size=nf, max_size=nf))
    gaps = draw(st.lists(st.integers(0, 40), min_size=nf, max_size=nf))
    kind = draw(st.sampled_from(["random", "runs", "zeros"]))
    seed = draw(st.integers(0, 2**32 - 1))
    return params, sizes, gaps, kind, seed


def materialize(sizes, gaps, kind, seed):
    rng = np.random.default_rng(seed)
    offs, pos = [], 0
    for n, g in zip(sizes, gaps):
        pos += g
        offs.append(pos)
        pos += n
    total = pos + int(rng.integers(0, 64))               # trailing slack (or none)
    if kind == "random":
        buf = rng.integers(0, 256, total, dtype=np.uint8)
    elif kind == "runs":
        sym = rng.integers(0, 256, 3, dtype=np.uint8)
        buf = np.repeat(sym[rng.integers(0, 3, total // 50 + 1)], 50)[:total].copy()
    else:
        buf = np.zeros(total, np.uint8)
    return buf, np.array(offs, np.uint64), np.array(sizes, np.uint64)


@settings(max_examples=60, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(batches())
def test_random_batches_vs_oracle(chunkers, case):
    (bits, mx, cap), sizes, gaps, kind, seed = case
    buf, offs, lens = materialize(sizes, gaps, kind, seed)
    ch = chunkers(bits, mx, cap)
    got = ch.batch_arrays(buf, offs, lens, hashed=True)
    assert len(got) == lens.size
    mode = O.MODE_PRODUCTION if cap else O.MODE_IDEAL
    ref = O.chunk_batch(buf, offs, lens, bits=bits, max_chunk=mx, read_cap=cap, mode=mode)
    o, n = [], []
    for f, (g, r) in enumerate(zip(got, ref)):
        ends = (g["offset"].astype(np.int64) + g["len"].astype(np.int64)).tolist()
        assert ends == r.astype(np.int64).tolist(), f"file {f}"
        assert (g["file"] == f).all()
        o += (g["offset"].astype(np.uint64) + offs[f]).tolist()
        n += g["len"].astype(np.uint64).tolist()
    if o:
        want = O.blake3_batch(buf, np.array(o, np.uint64), np.array(n, np.uint64), nthreads=8)
        have = np.concatenate([g["hash"] for g in got])
        assert np.array_equal(have, want)
