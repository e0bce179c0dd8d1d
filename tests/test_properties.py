"""Property tests of the CPU oracle (the reference's structural
invariants as properties; tests/chunking_test.rs pins no offsets).

Random byte strings, chunk_bits, max_chunk and read caps drawn by hypothesis:
- the literal loop (compute_file_chunks, file_operations.rs:721-788 / chunk_data,
  tests/chunking_test.rs:170-192) and the closed-form restatement agree;
- cuts cover the input contiguously from 0 (chunking_test.rs:46-73,110-167);
- no chunk exceeds max_chunk (:95-108);
- empty input -> no chunk (:37-43); repeated calls agree (:11-23);
- a cut depends only on the bytes before it: rewriting everything after a cut
  keeps the cuts up to it (:76-92, 195-233).
"""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import oracle as O

SETTINGS = settings(max_examples=150, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow])


@st.composite
def cases(draw):
    bits = draw(st.integers(1, 16))
    max_chunk = draw(st.sampled_from([1, 7, 64, 100, 1000, 4096, 1 << 16]))
    read_cap = draw(st.sampled_from([0, 1, 63, 64, 65, 1000, 4096]))
    kind = draw(st.sampled_from(["random", "runs", "zeros"]))
    n = draw(st.integers(0, 20000))
    seed = draw(st.integers(0, 2**32 - 1))
    rng = np.random.default_rng(seed)
    if kind == "random":
        data = rng.integers(0, 256, n, dtype=np.uint8)
    elif kind == "runs":                          # low-entropy: long runs of few symbols
        sym = rng.integers(0, 256, 4, dtype=np.uint8)
        data = np.repeat(sym[rng.integers(0, 4, n // 37 + 1)], 37)[:n].copy()
    else:
        data = np.zeros(n, np.uint8)
    return data, bits, max_chunk, read_cap


def check_structure(ends, n, max_chunk):
    ends = np.asarray(ends, dtype=np.int64)
    if n == 0:
        assert ends.size == 0
        return
    assert ends.size >= 1 and ends[-1] == n
    sizes = np.diff(np.concatenate([[0], ends]))
    assert (sizes >= 1).all() and (sizes <= max_chunk).all()


@SETTINGS
@given(cases())
def test_formulations_agree_and_structure(case):
    data, bits, mx, cap = case
    prod = O.chunk_production(data, bits, mx, cap if cap else 1 << 62)
    closed = O.chunk_closed_form(data, bits, mx, cap)
    ideal = O.chunk_ideal(data, bits, mx)
    assert np.array_equal(prod if cap else ideal, closed)
    check_structure(prod, data.size, mx)
    check_structure(ideal, data.size, mx)
    assert np.array_equal(O.chunk_production(data, bits, mx, cap if cap else 1 << 62), prod)   # determinism


@SETTINGS
@given(cases(), st.integers(0, 2**32 - 1))
def test_edit_after_a_cut_keeps_earlier_cuts(case, seed):
    data, bits, mx, cap = case
    ends = O.chunk_ideal(data, bits, mx)
    if ends.size < 2:
        return
    keep = int(ends[ends.size // 2 - 1])             # a cut in the first half
    edited = data.copy()
    rng = np.random.default_rng(seed)
    tail = edited[keep:]
    tail[:] = rng.integers(0, 256, tail.size, dtype=np.uint8)
    e2 = O.chunk_ideal(edited, bits, mx)
    assert e2[:ends.size // 2].tolist() == ends[:ends.size // 2].tolist()
