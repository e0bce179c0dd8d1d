"""Input recipes for golden fixtures (tests/golden/*.json).

A recipe regenerates the exact input bytes; fixtures never store raw blobs.
"chunking_test" recipes rebuild the inputs used by the reference's
tests/chunking_test.rs (byte patterns only, generated here).
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

_MAX13 = (1 << 13) * 16   # tests/chunking_test.rs:7-8


def _chunking_test_input(name: str) -> bytes:
    """Inputs of tests/chunking_test.rs (line refs for each)."""
    if name == "deterministic":          # :13
        return b"This is test content that will be chunked. " * 100
    if name == "small_file":             # :27
        return b"Small file"
    if name == "empty_file":             # :38
        return b""
    if name == "large_file":             # :48-56
        c = b"".join(b"Line %d with some varied content\n" % i for i in range(1000))
        while len(c) < 100 * 1024:
            c += b"Additional padding content to reach size. "
        return c
    if name == "content_shifting_1":     # :78-80
        return b"AAAAA" * 1000
    if name == "content_shifting_2":     # :82-84
        return b"PREFIX" + b"AAAAA" * 1000
    if name == "boundaries":             # :97
        return b"A" * (_MAX13 * 2)
    if name == "binary_data":            # :112
        return bytes(i % 256 for i in range(50000))
    if name == "identical_blocks":       # :124-125
        return b"IDENTICAL_BLOCK_CONTENT" * 500
    if name == "from_file":              # :141
        return b"Test data for chunking " * 1000
    if name == "offset_progression":     # :157
        return b"X" * 100000
    if name in ("modification_1", "modification_2"):   # :198-209
        return b"STABLE_PREFIX_" * 1000 + (b"_ENDING_1" if name.endswith("1") else b"_ENDING_2")
    raise KeyError(name)


def make_input(recipe: dict) -> np.ndarray:
    k = recipe["kind"]
    if k == "bytes":
        return np.frombuffer(bytes.fromhex(recipe["hex"]), dtype=np.uint8).copy()
    if k == "xorshift":
        d = O.xorshift_bytes(recipe["seed"], recipe["n"], recipe.get("discard", 0))
        if "zero" in recipe:
            a, b = recipe["zero"]
            d[a:b] = 0
        for a, b, byte in recipe.get("fill", []):          # constant runs (no hits: read-cap / MAX cuts)
            d[a:b] = byte
        for off, hx in recipe.get("patch", []):            # planted bytes (tests/golden/make_golden.py)
            p = np.frombuffer(bytes.fromhex(hx), dtype=np.uint8)
            d[off:off + p.size] = p
        return d
    if k == "const":
        return np.full(recipe["n"], recipe["byte"], np.uint8)
    if k == "chunking_test":
        return np.frombuffer(_chunking_test_input(recipe["name"]), dtype=np.uint8).copy()
    raise KeyError(k)
