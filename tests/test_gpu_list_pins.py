"""The reference's LIST-level chunk pins (tests/protocol_list_test.rs), end to end
on the GPU path: file on disk -> compute_file_chunks (GPU chunking + BLAKE3,
production semantics) -> LIST `C` lines (syncr_cdc_format_chunks, the text of
v3_server.rs:146-182) -> parsed back the way v3_client.rs:272-300 reads them.

- a 5-byte file is exactly one chunk (0, 5)               (:305-322)
- the chunk hash is stable across two LISTs               (:325-340)
- 50 MiB of 'A' is more than one chunk, exact coverage    (:360-378)
- 100 000 x 'X' has sequential offsets                    (:381-400)
- an empty file is listed with no chunks                  (:576-589)
"""
import base64
import json

import numpy as np
import pytest

import syncr_amd
from oracle import oracle as O

pytestmark = pytest.mark.gpu
M = 1 << 20


def list_chunks(path, ch):
    """LIST `C` lines of one file, parsed: [(off, len, hsh)]."""
    cs = syncr_amd.compute_file_chunks(str(path), ch, hashed=True)
    arr = np.zeros(len(cs), syncr_amd.CHUNK_INFO_DTYPE)
    for i, c in enumerate(cs):
        arr[i]["offset"], arr[i]["len"] = c.offset, c.size
        arr[i]["hash"] = np.frombuffer(bytes(c.hash), np.uint8)
    text = syncr_amd.format_chunks(arr, syncr_amd.FMT_LIST_LINES).decode()
    out = []
    for line in text.splitlines():
        j = json.loads(line)
        assert j["typ"] == "C"
        out.append((j["off"], j["len"], j["hsh"]))
    return out


@pytest.fixture(scope="module")
def ch():
    with syncr_amd.Chunker(syncr_amd.CHUNK_BITS, syncr_amd.MAX_CHUNK_SIZE, syncr_amd.TOKIO_READ_CAP) as c:
        yield c


def test_small_file_one_chunk_and_stable_hash(tmp_path, ch):
    p = tmp_path / "small.txt"
    p.write_bytes(b"small")
    first = list_chunks(p, ch)
    assert [(o, n) for o, n, _ in first] == [(0, 5)]
    assert first[0][2] == base64.urlsafe_b64encode(O.blake3(b"small")).decode()
    assert list_chunks(p, ch) == first


def test_large_uniform_file_exact_coverage(tmp_path, ch):
    p = tmp_path / "big.bin"
    p.write_bytes(b"A" * (50 * M))
    cs = list_chunks(p, ch)
    assert len(cs) > 1
    assert sum(n for _, n, _ in cs) == 50 * M
    assert [o for o, _, _ in cs] == [sum(n for _, n, _ in cs[:i]) for i in range(len(cs))]
    want = O.ends_to_cuts(O.chunk_production(np.full(50 * M, ord("A"), np.uint8)))
    assert [(o, n) for o, n, _ in cs] == want


def test_sequential_offsets(tmp_path, ch):
    p = tmp_path / "x.bin"
    p.write_bytes(b"X" * 100000)
    cs = list_chunks(p, ch)
    assert cs[0][0] == 0
    for (o, n, _), (o2, _, _) in zip(cs, cs[1:]):
        assert o2 == o + n
    assert cs[-1][0] + cs[-1][1] == 100000


def test_empty_file_no_chunks(tmp_path, ch):
    p = tmp_path / "empty"
    p.write_bytes(b"")
    assert list_chunks(p, ch) == []
