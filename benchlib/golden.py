"""Golden fixtures and per-file digests (the checker side of bench.py's parity
leg and of smoke()).  Test infrastructure: the digests of GPU results are
computed with the oracle's FNV helper and compared with fixtures the CPU
oracle produced (tests/golden/make_corpus_digests.py); nothing here is on the
measured path."""
from __future__ import annotations

import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

_cache: dict = {}


def load_digests(name: str) -> dict | None:
    """tests/golden/<name>_digests.npz (no pickles), or None if absent."""
    if name not in _cache:
        p = os.path.join(GOLDEN, f"{name}_digests.npz")
        _cache[name] = dict(np.load(p, allow_pickle=False)) if os.path.exists(p) else None
    return _cache[name]


def load_json(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def ends_of(c: np.ndarray) -> np.ndarray:
    """Cut END offsets (file-relative) of one file's structured cut array."""
    return c["offset"].astype(np.uint64) + c["len"].astype(np.uint64)


def file_digest(c: np.ndarray, hashed: bool = False) -> tuple[int, int, int | None]:
    from oracle import oracle as O
    return (int(c.size), O.fnv_ends(ends_of(c)), O.fnv_hashes(c["hash"]) if hashed else None)


def check_files(name: str, cuts: list, rows, semantics: str = "production", hashed: bool = False) -> dict:
    """Compare each file's GPU result with golden row rows[j] of fixture `name`.
    semantics: "production" (read_cap 2 MiB) or "ideal" (read_cap 0).  Rows
    outside the fixture (weak-scaled copies with other seeds) are skipped."""
    g = load_digests(name)
    if g is None:
        return {"fixture": f"tests/golden/{name}_digests.npz", "missing": True}
    pre = "" if semantics == "production" else "ideal_"
    nref, fref = g[pre + "nchunks"], g[pre + "ends_fnv"]
    href = g["hash_fnv"] if hashed else None
    files = chunks = bad = 0
    first = None
    rows = np.asarray(rows, dtype=np.int64)
    for j, r in enumerate(rows.tolist()):
        if r < 0 or r >= nref.size:
            continue
        n, fe, fh = file_digest(cuts[j], hashed)
        ok = n == int(nref[r]) and fe == int(fref[r]) and (href is None or fh == int(href[r]))
        files += 1
        chunks += n
        if not ok:
            bad += 1
            if first is None:
                first = {"file": int(r), "chunks": n, "want_chunks": int(nref[r])}
    out = {"files": files, "chunks": chunks, "mismatches": bad, "semantics": semantics,
           "hashes": bool(hashed), "fixture": f"tests/golden/{name}_digests.npz"}
    if first is not None:
        out["first_mismatch"] = first
    return out
