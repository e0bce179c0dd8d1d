"""CPU checks of the BLAKE3 oracle (oracle/blake3_oracle.c), the checker of the
GPU chunk hasher.  It restates blake3::hash as called by util::hash_binary
(reference src/util.rs:57-59) per chunk (src/protocol/file_operations.rs:757).

Pinned by the official BLAKE3 test vectors (tests/golden/blake3_vectors.json)
and by the reference's own util.rs tests (:77-135): 44-character base64,
determinism, distinct inputs -> distinct hashes."""
import json
import os

import numpy as np

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "blake3_vectors.json")


def vectors():
    return json.load(open(GOLDEN))


def test_official_vectors():
    v = vectors()
    for n, want in v["cases"]:
        data = (np.arange(n) % 251).astype(np.uint8)
        assert O.blake3(data).hex() == want, n
    for s, want in v["strings"]:
        assert O.blake3(s.encode()).hex() == want, s


def test_batch_matches_single():
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 300_000, dtype=np.uint8)
    offs = np.array([0, 1, 17, 1000, 5000, 123_456], np.uint64)
    lens = np.array([0, 1, 64, 1025, 100_000, 176_544], np.uint64)
    got = O.blake3_batch(buf, offs, lens, nthreads=3)
    for i in range(offs.size):
        o, n = int(offs[i]), int(lens[i])
        assert got[i].tobytes() == O.blake3(buf[o:o + n])


def test_reference_util_properties():
    """src/util.rs:77-135: 44 base64 chars, deterministic, distinct inputs differ."""
    for src in (b"12", b"", b"The quick brown fox jumps over the lazy dog", bytes([0, 0xFF, 0xDE, 0xAD])):
        b64 = O.hash_to_base64(O.blake3(src))
        assert len(b64) == 44 and b64 == O.hash_to_base64(O.blake3(src))
    assert O.blake3(b"test1") != O.blake3(b"test2")
    # URL_SAFE alphabet with padding (util.rs:62-64)
    assert O.hash_to_base64(bytes([0xfb] * 32)).endswith("=") and "+" not in O.hash_to_base64(bytes([0xfb] * 32))
