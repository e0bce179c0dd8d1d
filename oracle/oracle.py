"""ctypes front-end of the CPU oracle (oracle/bup_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the *checker*.  The product package
(syncr_amd) never imports this module.

Reference semantics restated (paths relative to /root/reference):
  * production driver  src/protocol/file_operations.rs:721-788
  * ideal driver       tests/chunking_test.rs:170-192
  * parameters         src/chunking.rs:7-13
  * rollsum::Bup       rollsum 0.3 (Cargo.toml:24; crate not on disk)
  * util::hash_binary  blake3::hash, blake3 1.8 (Cargo.toml:14; crate not on disk),
                       src/util.rs:57-59, restated in oracle/blake3_oracle.c
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc_bup.so")

CHUNK_BITS = 20                       # src/chunking.rs:7
MAX_CHUNK_SIZE = (1 << 20) * 16       # src/chunking.rs:10-13
TOKIO_READ_CAP = 2 * 1024 * 1024      # tokio DEFAULT_MAX_BUF_SIZE (Cargo.toml:29)

MODE_PRODUCTION, MODE_IDEAL, MODE_CLOSED_FORM, MODE_PRODUCTION_WINDOW = 0, 1, 2, 3

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build() -> str:
    """Compile liborc_bup.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(os.path.join(_HERE, f))
                                              for f in ("bup_oracle.c", "blake3_oracle.c"))
        ):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_chunk_production.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                           ctypes.c_uint64, _u64p, ctypes.c_uint64]
        L.orc_chunk_production.restype = ctypes.c_uint64
        L.orc_chunk_production_window.argtypes = L.orc_chunk_production.argtypes
        L.orc_chunk_production_window.restype = ctypes.c_uint64
        L.orc_chunk_closed_form.argtypes = L.orc_chunk_production.argtypes
        L.orc_chunk_closed_form.restype = ctypes.c_uint64
        L.orc_chunk_no_head_fixup.argtypes = L.orc_chunk_production.argtypes
        L.orc_chunk_no_head_fixup.restype = ctypes.c_uint64
        L.orc_chunk_production_read_error.argtypes = L.orc_chunk_production.argtypes
        L.orc_chunk_production_read_error.restype = ctypes.c_uint64
        L.orc_chunk_ideal.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                      _u64p, ctypes.c_uint64]
        L.orc_chunk_ideal.restype = ctypes.c_uint64
        L.orc_digest_after.argtypes = [_u8p, ctypes.c_uint64]
        L.orc_digest_after.restype = ctypes.c_uint32
        L.orc_xorshift_fill.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _u8p, ctypes.c_uint64]
        L.orc_xorshift_fill.restype = None
        L.orc_corpus_seed.argtypes = [ctypes.c_uint64]
        L.orc_corpus_seed.restype = ctypes.c_uint64
        L.orc_corpus_fill.argtypes = [_u64p, _u64p, ctypes.c_uint64, ctypes.c_uint64, _u8p]
        L.orc_corpus_fill.restype = None
        L.orc_fnv_ends.argtypes = [_u64p, ctypes.c_uint64]
        L.orc_fnv_ends.restype = ctypes.c_uint64
        L.orc_chunk_batch.argtypes = [_u8p, _u64p, _u64p, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, _u64p, _u64p,
                                      _u64p, _u64p, ctypes.c_int]
        L.orc_chunk_batch.restype = ctypes.c_int
        L.orc_blake3.argtypes = [_u8p, ctypes.c_uint64, _u8p]
        L.orc_blake3.restype = None
        L.orc_blake3_batch.argtypes = [_u8p, _u64p, _u64p, ctypes.c_uint64, _u8p, ctypes.c_int]
        L.orc_blake3_batch.restype = ctypes.c_int
        _lib = L
    return _lib


def _p8(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def _p64(a: np.ndarray):
    return a.ctypes.data_as(_u64p)


def _as_u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8)


def _run(fn, data, *args) -> np.ndarray:
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    cap = max(16, a.size // 4096 + 64)
    while True:
        ends = np.zeros(cap, np.uint64)
        n = fn(_p8(buf), a.size, *args, _p64(ends), cap)
        if n == 2**64 - 1:
            raise MemoryError("oracle allocation failed")
        if n <= cap:
            return ends[:n].copy()
        cap = int(n)


def chunk_production(data, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE, read_cap=TOKIO_READ_CAP):
    """Cut END offsets of compute_file_chunks (file_operations.rs:721-788)."""
    return _run(lib().orc_chunk_production, data, bits, max_chunk, read_cap)


def chunk_production_read_error(data, P, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE, read_cap=TOKIO_READ_CAP):
    """Cut ends compute_file_chunks keeps when every read at file offset >= P
    fails (file_operations.rs:738-743 for P = 0, :776-782 otherwise); only
    data[:P] is ever read (bup_oracle.c orc_chunk_production_read_error)."""
    return _run(lib().orc_chunk_production_read_error, _as_u8(data)[:P], bits, max_chunk, read_cap)


def chunk_production_window(data, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE, read_cap=TOKIO_READ_CAP):
    """The literal loop without copy_within's memmove (buffer = window into the
    file): same reads, same Bup state machine, same cuts; for inputs with very
    many chunks (bup_oracle.c orc_chunk_production_window)."""
    return _run(lib().orc_chunk_production_window, data, bits, max_chunk, read_cap)


def chunk_ideal(data, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE):
    """Cut END offsets of chunk_data (tests/chunking_test.rs:170-192)."""
    return _run(lib().orc_chunk_ideal, data, bits, max_chunk)


def chunk_closed_form(data, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE, read_cap=TOKIO_READ_CAP):
    """Formulation (ii): prefix-sum candidates + serial resolve (read_cap=0: ideal)."""
    return _run(lib().orc_chunk_closed_form, data, bits, max_chunk, read_cap)


def chunk_no_head_fixup(data, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE, read_cap=TOKIO_READ_CAP):
    """Deliberately wrong (no chunk-head fix-up): adversarial-input search only."""
    return _run(lib().orc_chunk_no_head_fixup, data, bits, max_chunk, read_cap)


def ends_to_cuts(ends) -> list[tuple[int, int]]:
    """[(offset, size)] like the reference's ChunkInfo{offset,size} (protocol/types.rs:24-29)."""
    out, prev = [], 0
    for e in np.asarray(ends, dtype=np.uint64).tolist():
        out.append((prev, e - prev))
        prev = e
    return out


def digest_after(data) -> int:
    a = _as_u8(data)
    return int(lib().orc_digest_after(_p8(a if a.size else np.zeros(1, np.uint8)), a.size))


def xorshift_bytes(seed: int, n: int, discard: int = 0) -> np.ndarray:
    out = np.empty(max(n, 1), np.uint8)
    lib().orc_xorshift_fill(seed, discard, _p8(out), n)
    return out[:n]


def corpus_seed(i: int) -> int:
    return int(lib().orc_corpus_seed(i))


def corpus_fill(lens, first_index: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Back-to-back corpus of xorshift files. Returns (bytes, offsets)."""
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    offs = np.zeros_like(lens)
    if lens.size:
        offs[1:] = np.cumsum(lens)[:-1]
    total = int(lens.sum())
    buf = np.empty(max(total, 1), np.uint8)
    lib().orc_corpus_fill(_p64(offs), _p64(lens), lens.size, first_index, _p8(buf))
    return buf[:total], offs


def corpus_fill_threads(lens, indices=None, nthreads: int = 8) -> tuple[np.ndarray, np.ndarray]:
    """corpus_fill with file j = corpus file indices[j] (default j), on threads."""
    from concurrent.futures import ThreadPoolExecutor
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    idx = np.arange(lens.size, dtype=np.uint64) if indices is None else np.ascontiguousarray(indices, np.uint64)
    offs = np.zeros_like(lens)
    if lens.size:
        offs[1:] = np.cumsum(lens)[:-1]
    total = int(lens.sum())
    buf = np.empty(max(total, 1), np.uint8)
    L = lib()

    def one(j):
        o, n = offs[j:j + 1], lens[j:j + 1]
        L.orc_corpus_fill(_p64(o), _p64(n), 1, int(idx[j]), _p8(buf))

    order = np.argsort(-lens.astype(np.int64), kind="stable").tolist()
    with ThreadPoolExecutor(nthreads) as ex:
        list(ex.map(one, order))
    return buf[:total], offs


def fnv_ends(ends) -> int:
    e = np.ascontiguousarray(ends, dtype=np.uint64)
    return int(lib().orc_fnv_ends(_p64(e if e.size else np.zeros(1, np.uint64)), e.size))


def fnv_hashes(hashes) -> int:
    """FNV-1a-64 (orc_fnv_ends) over a file's chunk hashes, [n, 32] uint8, read
    as 4 little-endian u64 words per hash: the per-file hash digest of the
    golden corpus fixtures (tests/golden/make_corpus_digests.py)."""
    h = np.ascontiguousarray(hashes, dtype=np.uint8).reshape(-1)
    return fnv_ends(h.view("<u8") if h.size else np.zeros(0, np.uint64))


def chunk_batch(base, offs, lens, bits=CHUNK_BITS, max_chunk=MAX_CHUNK_SIZE,
                read_cap=TOKIO_READ_CAP, mode=MODE_PRODUCTION, nthreads=None):
    """Chunk many files (threads over files, largest first). Returns list of end arrays."""
    base = _as_u8(base)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    n = lens.size
    caps = lens // max(1, 1 << max(0, bits - 6)) + 64
    order = np.argsort(-lens.astype(np.int64), kind="stable")
    ob = np.zeros(n, np.uint64)
    if n:
        ob[1:] = np.cumsum(caps)[:-1]
    ends = np.zeros(max(int(caps.sum()), 1), np.uint64)
    counts = np.zeros(max(n, 1), np.uint64)
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    # pass the permuted tables so big files start first
    po, pl, pb, pc = (np.ascontiguousarray(a[order]) for a in (offs, lens, ob, caps))
    pcount = np.zeros(max(n, 1), np.uint64)
    lib().orc_chunk_batch(_p8(base if base.size else np.zeros(1, np.uint8)), _p64(po), _p64(pl), n,
                          bits, max_chunk, read_cap, mode, _p64(pb), _p64(pc), _p64(ends),
                          _p64(pcount), nthreads)
    counts[order] = pcount[:n]
    out = []
    for i in range(n):
        c = int(counts[i])
        if c > int(caps[i]):  # rare: re-run this file alone with exact capacity
            f = base[int(offs[i]): int(offs[i]) + int(lens[i])]
            fn = {MODE_PRODUCTION: chunk_production, MODE_CLOSED_FORM: chunk_closed_form,
                  MODE_PRODUCTION_WINDOW: chunk_production_window}.get(mode)
            out.append(chunk_ideal(f, bits, max_chunk) if mode == MODE_IDEAL else fn(f, bits, max_chunk, read_cap))
        else:
            out.append(ends[int(ob[i]): int(ob[i]) + c].copy())
    return out


def blake3(data) -> bytes:
    """blake3::hash(data) (util::hash_binary, src/util.rs:57-59)."""
    a = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8) if not isinstance(data, np.ndarray) \
        else np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    out = np.zeros(32, np.uint8)
    buf = a if a.size else np.zeros(1, np.uint8)
    lib().orc_blake3(_p8(buf), a.size, _p8(out))
    return out.tobytes()


def blake3_batch(base: np.ndarray, offs, lens, nthreads: int = 1) -> np.ndarray:
    """[n, 32] uint8: blake3 of base[offs[i] : offs[i] + lens[i]] for every i."""
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    out = np.zeros((offs.size, 32), np.uint8)
    buf = base if base.size else np.zeros(1, np.uint8)
    rc = lib().orc_blake3_batch(_p8(buf), offs.ctypes.data_as(_u64p), lens.ctypes.data_as(_u64p),
                                offs.size, out.ctypes.data_as(_u8p), nthreads)
    if rc:
        raise RuntimeError("orc_blake3_batch failed")
    return out


def hash_to_base64(h: bytes) -> str:
    """util::hash_to_base64: base64 URL_SAFE with padding (src/util.rs:62-64)."""
    import base64
    return base64.urlsafe_b64encode(h).decode()
