"""syncr_amd -- MI355X-native Bup content-defined chunker (host mirror).

Python mirror of szilu/syncr's chunking interface over the C ABI in
include/syncr_cdc.h (libsyncr_cdc.so, HIP kernels for gfx950):

  * constants             src/chunking.rs:7-13           -> CHUNK_BITS, MAX_CHUNK_SIZE
  * ChunkInfo             src/protocol/types.rs:24-29    -> ChunkInfo(offset, size, hash)
  * compute_file_chunks   src/protocol/file_operations.rs:721-788
                          (open/read failure -> warn + empty list, like :727-744)
  * chunk_data            tests/chunking_test.rs:170-192 (ideal, in-memory semantics)

There is no CPU fallback: if the HIP library is missing or no GPU is visible the
calls raise (SyncrCdcError), they never silently compute on the host.
"""
from __future__ import annotations

import ctypes
import logging
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

__all__ = [
    "CHUNK_BITS", "MAX_CHUNK_SIZE_FACTOR", "MAX_CHUNK_SIZE", "TOKIO_READ_CAP",
    "ChunkInfo", "Chunker", "ChunkCache", "Ingest", "SyncrCdcError", "format_chunks", "compute_file_chunks", "chunk_data",
    "library", "library_path", "EXPORTED_SYMBOLS",
]

log = logging.getLogger("syncr_amd")

CHUNK_BITS = 20                                   # src/chunking.rs:7
MAX_CHUNK_SIZE_FACTOR = 16                        # src/chunking.rs:10
MAX_CHUNK_SIZE = (1 << CHUNK_BITS) * MAX_CHUNK_SIZE_FACTOR   # src/chunking.rs:13
TOKIO_READ_CAP = 2 * 1024 * 1024                  # tokio File::read (file_operations.rs:738,776)

_PKG = os.path.dirname(os.path.abspath(__file__))
library_path = os.path.join(_PKG, "libsyncr_cdc.so")

# every symbol declared in include/syncr_cdc.h
EXPORTED_SYMBOLS = (
    "syncr_cdc_abi_version", "syncr_cdc_strerror", "syncr_cdc_default_params",
    "syncr_cdc_device_count", "syncr_cdc_open", "syncr_cdc_close", "syncr_cdc_get_params",
    "syncr_cdc_chunk_host", "syncr_cdc_chunk_batch_host", "syncr_cdc_plan", "syncr_cdc_launch",
    "syncr_cdc_fetch", "syncr_cdc_chunk_batch_device", "syncr_cdc_device_alloc",
    "syncr_cdc_device_free", "syncr_cdc_host_alloc_pinned", "syncr_cdc_host_free_pinned",
    "syncr_cdc_memcpy_h2d", "syncr_cdc_memcpy_d2h", "syncr_cdc_memcpy_d2d", "syncr_cdc_synchronize", "syncr_cdc_stream",
    "syncr_cdc_gen_corpus", "syncr_cdc_read_probe", "syncr_cdc_set_timing", "syncr_cdc_kernel_times",
    "syncr_cdc_last_stats", "syncr_cdc_split_stats", "syncr_cdc_get_info",
    "syncr_cdc_chunk_host_hashed", "syncr_cdc_chunk_batch_host_hashed", "syncr_cdc_launch_hashed",
    "syncr_cdc_fetch_hashed", "syncr_cdc_kernel_times_ex",
    "syncr_cdc_format_chunks",
    "syncr_ingest_open", "syncr_ingest_submit", "syncr_ingest_submit_file", "syncr_ingest_reserve",
    "syncr_ingest_commit", "syncr_ingest_flush", "syncr_ingest_stats", "syncr_ingest_close",
    "syncr_cache_open", "syncr_cache_get", "syncr_cache_put", "syncr_cache_sync", "syncr_cache_stats",
    "syncr_cache_close", "syncr_ingest_set_cache", "syncr_ingest_cache_hits",
    "syncr_ingest_open_multi", "syncr_ingest_device_stats", "syncr_cache_get_params",
    "syncr_ingest_set_read_fault", "syncr_cdc_fetch_reruns", "syncr_ingest_timing",
    "syncr_cdc_last_scan",
)

ABI_VERSION = 3
E_RANGE = -34
E_NOENT = -2
E_BUSY = -16
E_INVAL = -22
FLAG_RESOLVE_LANE = 1       # exact alternative resolves (include/syncr_cdc.h SYNCR_CDC_FLAG_*)
FLAG_RESOLVE_NOBURST = 2
FLAG_RESOLVE_NOSPLIT = 4
FLAG_SPLIT_NOWAIT = 8       # testing: split-walk workers give up at once
FMT_LIST_LINES = 1      # LIST reply "C" lines (src/protocol/v3_server.rs:146-182)
FMT_HASHCHUNKS = 2      # profile FileData "ch" array (src/types.rs:117-129)


class SyncrCdcError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        msg = library().syncr_cdc_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})")


class Params(ctypes.Structure):
    _fields_ = [("chunk_bits", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("max_chunk", ctypes.c_uint64), ("read_cap", ctypes.c_uint64)]


class Cut(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("len", ctypes.c_uint32), ("file", ctypes.c_uint32)]


CUT_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("file", "<u4")])
assert CUT_DTYPE.itemsize == ctypes.sizeof(Cut) == 16
# syncr_chunk_info: ChunkInfo{hash, offset, size} + file (include/syncr_cdc.h)
CHUNK_INFO_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("file", "<u4"), ("hash", "u1", (32,))])
assert CHUNK_INFO_DTYPE.itemsize == 48

_lib = None
_vp, _u64, _u32, _i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32
_pu64 = ctypes.POINTER(ctypes.c_uint64)
# syncr_ingest_cb(ctx, tag, status, const syncr_chunk_info *chunks, n)
_INGEST_CB = ctypes.CFUNCTYPE(None, _vp, _u64, _i32, _vp, _u64)


def use_dev_library() -> None:
    """tools/ only: load libsyncr_cdc_dev.so (python -m syncr_amd.build --dev)
    instead of the product library.  It adds scan variants and timing-only
    ablations chosen by SYNCR_CDC_* / SYNCR_B3_* environment variables; the
    product library reads no environment.  Must run before the first library()."""
    global library_path
    if _lib is not None:
        raise RuntimeError("syncr_amd: library already loaded")
    library_path = os.path.join(_PKG, "libsyncr_cdc_dev.so")


def library():
    """Load libsyncr_cdc.so (raises if it was not built -- no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(library_path):
            raise ImportError(f"syncr_amd: {library_path} not built; run `python -m syncr_amd.build` "
                              "(the HIP engine has no CPU fallback)")
        L = ctypes.CDLL(library_path)
        sig = {
            "syncr_cdc_abi_version": ([], _i32),
            "syncr_cdc_strerror": ([_i32], ctypes.c_char_p),
            "syncr_cdc_default_params": ([ctypes.POINTER(Params)], None),
            "syncr_cdc_device_count": ([ctypes.POINTER(_i32)], _i32),
            "syncr_cdc_open": ([_i32, ctypes.POINTER(Params), ctypes.POINTER(_vp)], _i32),
            "syncr_cdc_close": ([_vp], None),
            "syncr_cdc_get_params": ([_vp, ctypes.POINTER(Params)], _i32),
            "syncr_cdc_chunk_host": ([_vp, _vp, _u64, _vp, _u64, _pu64], _i32),
            "syncr_cdc_chunk_batch_host": ([_vp, _vp, _u64, _vp, _vp, _u32, _vp, _u64, _vp, _pu64], _i32),
            "syncr_cdc_plan": ([_vp, _vp, _vp, _u32, _u64], _i32),
            "syncr_cdc_launch": ([_vp, _vp, _vp], _i32),
            "syncr_cdc_fetch": ([_vp, _vp, _u64, _vp, _pu64], _i32),
            "syncr_cdc_chunk_batch_device": ([_vp, _vp, _u64, _vp, _vp, _u32, _vp, _u64, _vp, _pu64, _vp], _i32),
            "syncr_cdc_device_alloc": ([_vp, _u64, ctypes.POINTER(_vp)], _i32),
            "syncr_cdc_device_free": ([_vp, _vp], _i32),
            "syncr_cdc_host_alloc_pinned": ([_vp, _u64, ctypes.POINTER(_vp)], _i32),
            "syncr_cdc_host_free_pinned": ([_vp, _vp], _i32),
            "syncr_cdc_memcpy_h2d": ([_vp, _vp, _vp, _u64, _vp], _i32),
            "syncr_cdc_memcpy_d2h": ([_vp, _vp, _vp, _u64, _vp], _i32),
            "syncr_cdc_memcpy_d2d": ([_vp, _vp, _vp, _u64, _vp], _i32),
            "syncr_cdc_synchronize": ([_vp], _i32),
            "syncr_cdc_stream": ([_vp], _vp),
            "syncr_cdc_gen_corpus": ([_vp, _vp, _vp, _vp, _vp, _u32, _u64, _vp], _i32),
            "syncr_cdc_read_probe": ([_vp, _vp, _u64, _u32, _i32, ctypes.POINTER(ctypes.c_double)], _i32),
            "syncr_cdc_set_timing": ([_vp, _i32], _i32),
            "syncr_cdc_kernel_times": ([_vp, ctypes.POINTER(ctypes.c_double), _pu64], _i32),
            "syncr_cdc_last_stats": ([_vp, _pu64], _i32),
            "syncr_cdc_split_stats": ([_vp, _pu64], _i32),
            "syncr_cdc_fetch_reruns": ([_vp, _pu64], _i32),
            "syncr_cdc_get_info": ([_vp, _pu64], _i32),
            "syncr_cdc_last_scan": ([_vp, _pu64, ctypes.POINTER(ctypes.c_char_p)], _i32),
            "syncr_cdc_chunk_host_hashed": ([_vp, _vp, _u64, _vp, _u64, _pu64], _i32),
            "syncr_cdc_chunk_batch_host_hashed": ([_vp, _vp, _u64, _vp, _vp, _u32, _vp, _u64, _vp, _pu64], _i32),
            "syncr_cdc_launch_hashed": ([_vp, _vp, _vp], _i32),
            "syncr_cdc_fetch_hashed": ([_vp, _vp, _u64, _vp, _pu64], _i32),
            "syncr_cdc_kernel_times_ex": ([_vp, ctypes.POINTER(ctypes.c_double), _u32, _pu64], _i32),
            "syncr_cdc_format_chunks": ([_vp, _u64, _i32, _vp, _u64, _pu64], _i32),
            "syncr_ingest_open": ([_i32, ctypes.POINTER(Params), _u64, _u32, _u32, _INGEST_CB, _vp,
                                   ctypes.POINTER(_vp)], _i32),
            "syncr_ingest_submit": ([_vp, _vp, _u64, _u64], _i32),
            "syncr_ingest_submit_file": ([_vp, ctypes.c_char_p, _u64], _i32),
            "syncr_ingest_reserve": ([_vp, _u64, ctypes.POINTER(_vp)], _i32),
            "syncr_ingest_commit": ([_vp, _u64], _i32),
            "syncr_ingest_flush": ([_vp], _i32),
            "syncr_ingest_stats": ([_vp, _pu64], _i32),
            "syncr_ingest_close": ([_vp], None),
            "syncr_cache_open": ([ctypes.c_char_p, ctypes.POINTER(Params), ctypes.POINTER(_vp)], _i32),
            "syncr_cache_get_params": ([_vp, ctypes.POINTER(Params)], _i32),
            "syncr_ingest_open_multi": ([ctypes.POINTER(_i32), _u32, ctypes.POINTER(Params), _u64, _u32, _u32,
                                         _INGEST_CB, _vp, ctypes.POINTER(_vp)], _i32),
            "syncr_ingest_device_stats": ([_vp, _pu64, _u32], _i32),
            "syncr_ingest_set_read_fault": ([_vp, _u64, _i32], _i32),
            "syncr_ingest_timing": ([_vp, ctypes.POINTER(ctypes.c_double), _u32], _i32),
            "syncr_cache_get": ([_vp, ctypes.c_char_p, _u32, _u64, _vp, _u64, _pu64], _i32),
            "syncr_cache_put": ([_vp, ctypes.c_char_p, _u32, _u64, _vp, _u64], _i32),
            "syncr_cache_sync": ([_vp], _i32),
            "syncr_cache_stats": ([_vp, _pu64], _i32),
            "syncr_cache_close": ([_vp], None),
            "syncr_ingest_set_cache": ([_vp, _vp], _i32),
            "syncr_ingest_cache_hits": ([_vp, _pu64], _i32),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.syncr_cdc_abi_version() != ABI_VERSION:
            raise ImportError("syncr_amd: ABI version mismatch with libsyncr_cdc.so")
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise SyncrCdcError(rc, what)


def device_count() -> int:
    n = ctypes.c_int32(0)
    rc = library().syncr_cdc_device_count(ctypes.byref(n))
    return int(n.value) if rc == 0 else 0


@dataclass(frozen=True)
class ChunkInfo:
    """ChunkInfo{hash, offset, size} (src/protocol/types.rs:24-29).

    `hash` is BLAKE3 (util::hash_binary, src/util.rs:57-59) of the chunk's
    bytes, as in compute_file_chunks (file_operations.rs:757); None when the
    boundaries were requested without hashes."""
    offset: int
    size: int
    hash: Optional[bytes] = None


def _u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


# syncr_cdc_last_scan kinds (include/syncr_cdc.h SYNCR_CDC_SCAN_*)
SCAN_KINDS = {0: "none", 1: "stream_tiles", 2: "cu_schedule", 3: "tiles_dynamic", 255: "dev"}


class Chunker:
    """One engine handle on one device (Bup::new_with_chunk_bits, fixed params)."""

    def __init__(self, chunk_bits: int = CHUNK_BITS, max_chunk: int = MAX_CHUNK_SIZE,
                 read_cap: int = TOKIO_READ_CAP, device: int = 0, flags: int = 0):
        L = library()
        self.params = Params(chunk_bits, flags, max_chunk, read_cap)
        h = _vp()
        _check(L.syncr_cdc_open(device, ctypes.byref(self.params), ctypes.byref(h)), "syncr_cdc_open")
        self._h = h
        self.device = device
        self._nfiles = 0

    # -- lifetime ---------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            library().syncr_cdc_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return library().syncr_cdc_stream(self._h) or 0

    # -- host-memory paths ------------------------------------------------
    def cut_array(self, data) -> np.ndarray:
        """One file from host memory -> structured array (offset, len, file)."""
        a = _u8(data)
        return self.batch_arrays(a, [0], [a.size])[0]

    def chunk_bytes(self, data, hashed: bool = False) -> list[ChunkInfo]:
        """compute_file_chunks' ChunkInfo list for one file's bytes; with
        hashed=True each chunk carries its BLAKE3 hash (computed on the GPU)."""
        a = _u8(data)
        cuts = self.batch_arrays(a, [0], [a.size], hashed=hashed)[0]
        if hashed:
            return [ChunkInfo(int(c["offset"]), int(c["len"]), bytes(c["hash"])) for c in cuts]
        return [ChunkInfo(int(o), int(n)) for o, n, _ in cuts.tolist()]

    def batch_arrays(self, buf, offsets: Sequence[int], lengths: Sequence[int],
                     hashed: bool = False) -> list[np.ndarray]:
        L = library()
        a = _u8(buf)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        nf = offs.size
        counts = np.zeros(max(nf, 1), np.uint64)
        n = ctypes.c_uint64(0)
        cap = max(16, a.size // (1 << max(0, self.params.chunk_bits - 2)) + 4 * nf + 16)
        fn = L.syncr_cdc_chunk_batch_host_hashed if hashed else L.syncr_cdc_chunk_batch_host
        for _ in range(3):
            out = np.zeros(cap, CHUNK_INFO_DTYPE if hashed else CUT_DTYPE)
            rc = fn(self._h, a.ctypes.data if a.size else None, a.size, offs.ctypes.data, lens.ctypes.data,
                    nf, out.ctypes.data, cap, counts.ctypes.data, ctypes.byref(n))
            if rc == E_RANGE:
                cap = int(n.value)
                continue
            _check(rc, "syncr_cdc_chunk_batch_host" + ("_hashed" if hashed else ""))
            break
        return _split(out[: int(n.value)], counts[:nf])

    # -- device-resident paths (what the metric times) -------------------
    def plan(self, offsets, lengths, span: int) -> None:
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        _check(library().syncr_cdc_plan(self._h, offs.ctypes.data, lens.ctypes.data, offs.size, span),
               "syncr_cdc_plan")
        self._nfiles = offs.size

    def launch(self, d_bytes: int, stream: int = 0, hashed: bool = False) -> None:
        """Asynchronous scan + resolve (+ BLAKE3 of every chunk when hashed)."""
        fn = library().syncr_cdc_launch_hashed if hashed else library().syncr_cdc_launch
        _check(fn(self._h, d_bytes, stream or None), "syncr_cdc_launch" + ("_hashed" if hashed else ""))

    def fetch(self, hashed: bool = False) -> list[np.ndarray]:
        """Per-file structured arrays (offset, len, file[, hash])."""
        L = library()
        fn = L.syncr_cdc_fetch_hashed if hashed else L.syncr_cdc_fetch
        nf = self._nfiles
        counts = np.zeros(max(nf, 1), np.uint64)
        n = ctypes.c_uint64(0)
        rc = fn(self._h, None, 0, counts.ctypes.data, ctypes.byref(n))
        if rc not in (0, E_RANGE):
            _check(rc, "syncr_cdc_fetch")
        out = np.zeros(max(int(n.value), 1), CHUNK_INFO_DTYPE if hashed else CUT_DTYPE)
        _check(fn(self._h, out.ctypes.data, out.size, counts.ctypes.data, ctypes.byref(n)), "syncr_cdc_fetch")
        return _split(out[: int(n.value)], counts[:nf])

    def set_timing(self, on: bool, scan_only: bool = False, events: bool = False) -> None:
        """Per-kernel timing (syncr_cdc_set_timing): HIP events around each launch's
        phases; scan_only: the scan kernel alone, by the device clock (no queue
        packets), or with events=True by HIP events bound to its dispatch."""
        mode = ((2 if events else 4) if scan_only else 1) if on else 0
        _check(library().syncr_cdc_set_timing(self._h, mode), "syncr_cdc_set_timing")

    def kernel_times(self) -> tuple[list[float], int]:
        """Summed ms of [scan, dense+compaction, resolve, hash] since set_timing(True)."""
        ms = (ctypes.c_double * 4)()
        n = ctypes.c_uint64(0)
        _check(library().syncr_cdc_kernel_times_ex(self._h, ms, 4, ctypes.byref(n)), "syncr_cdc_kernel_times_ex")
        return [ms[0], ms[1], ms[2], ms[3]], int(n.value)

    def read_probe(self, d_ptr: int, nbytes: int, reps: int = 10, nt: bool = True) -> tuple[float, float]:
        """Streaming-read microbenchmark over device bytes: (best, mean) ms per pass."""
        ms = (ctypes.c_double * 2)()
        _check(library().syncr_cdc_read_probe(self._h, d_ptr, nbytes, reps, 1 if nt else 0, ms),
               "syncr_cdc_read_probe")
        return ms[0], ms[1]

    def last_stats(self) -> dict:
        st = (ctypes.c_uint64 * 4)()
        _check(library().syncr_cdc_last_stats(self._h, st), "syncr_cdc_last_stats")
        return {"candidates": st[0], "dense_tiles": st[1], "tiles": st[2], "flags": st[3]}

    def fetch_reruns(self) -> int:
        """Capacity re-runs the last fetch performed (syncr_cdc_fetch_reruns)."""
        n = ctypes.c_uint64(0)
        _check(library().syncr_cdc_fetch_reruns(self._h, ctypes.byref(n)), "syncr_cdc_fetch_reruns")
        return int(n.value)

    def split_stats(self) -> dict:
        """Split walks of long files in the last fetched launch (syncr_cdc_split_stats)."""
        st = (ctypes.c_uint64 * 6)()
        _check(library().syncr_cdc_split_stats(self._h, st), "syncr_cdc_split_stats")
        return dict(zip(("workers", "files_split", "segments", "walked", "adopted", "giveups"),
                        (int(x) for x in st)))

    def info(self) -> dict:
        v = (ctypes.c_uint64 * 8)()
        _check(library().syncr_cdc_get_info(self._h, v), "syncr_cdc_get_info")
        keys = ("run_bytes", "tile_bytes", "scan_grid", "compute_units", "scan_blocks_per_cu",
                "lds_bytes_per_scan_block", "device", "abi_version")
        return {k: int(x) for k, x in zip(keys, v)}

    def last_scan(self) -> dict:
        """The scan kernel the library ran for the last launch (syncr_cdc_last_scan):
        its own choice, never restated on this side."""
        v = (ctypes.c_uint64 * 4)()
        name = ctypes.c_char_p()
        _check(library().syncr_cdc_last_scan(self._h, v, ctypes.byref(name)), "syncr_cdc_last_scan")
        return {"kind": SCAN_KINDS.get(int(v[0]), str(int(v[0]))), "kernel": (name.value or b"").decode(),
                "tiles": int(v[1]), "waves": int(v[2]),
                "tiles_per_wave": round(int(v[1]) / int(v[2]), 3) if int(v[2]) else 0.0,
                "st_segments": int(v[3])}

    def synchronize(self) -> None:
        _check(library().syncr_cdc_synchronize(self._h), "syncr_cdc_synchronize")


class DeviceBuffer:
    """Device allocation owned by a Chunker's device (plumbing for tests/bench)."""

    def __init__(self, chunker: Chunker, nbytes: int):
        self._c = chunker
        p = _vp()
        _check(library().syncr_cdc_device_alloc(chunker.handle, nbytes, ctypes.byref(p)), "device_alloc")
        self.ptr = int(p.value)
        self.nbytes = nbytes

    def upload(self, data, offset: int = 0) -> None:
        a = _u8(data)
        if a.size:
            _check(library().syncr_cdc_memcpy_h2d(self._c.handle, self.ptr + offset, a.ctypes.data,
                                                  a.size, None), "memcpy_h2d")
            self._c.synchronize()

    def download(self, nbytes: Optional[int] = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(max(n, 1), np.uint8)
        if n:
            _check(library().syncr_cdc_memcpy_d2h(self._c.handle, out.ctypes.data, self.ptr + offset, n,
                                                  None), "memcpy_d2h")
            self._c.synchronize()
        return out[:n]

    def copy_from(self, src_ptr: int, nbytes: int, offset: int = 0) -> None:
        """Asynchronous device-to-device copy of nbytes at src_ptr to offset
        (on the chunker's stream; synchronize() before reading the result)."""
        if nbytes:
            _check(library().syncr_cdc_memcpy_d2d(self._c.handle, self.ptr + offset, src_ptr, nbytes, None),
                   "memcpy_d2d")

    def gen_corpus(self, offsets, lengths, first_index: int = 0, indices=None) -> None:
        """Synthetic corpus on the device: file i gets corpus file number
        indices[i] (default first_index + i)."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        idx = None if indices is None else np.ascontiguousarray(indices, dtype=np.uint64)
        _check(library().syncr_cdc_gen_corpus(self._c.handle, self.ptr, offs.ctypes.data, lens.ctypes.data,
                                              None if idx is None else idx.ctypes.data, offs.size,
                                              first_index, None), "gen_corpus")

    def free(self) -> None:
        if self.ptr:
            library().syncr_cdc_device_free(self._c.handle, self.ptr)
            self.ptr = 0


def format_chunks(chunks: np.ndarray, fmt: int = FMT_LIST_LINES) -> bytes:
    """Reference wire/on-disk text of a ChunkInfo list (CHUNK_INFO_DTYPE array):
    LIST reply lines or the profile's HashChunk array (syncr_cdc_format_chunks)."""
    a = np.ascontiguousarray(chunks, dtype=CHUNK_INFO_DTYPE)
    n = ctypes.c_uint64(0)
    rc = library().syncr_cdc_format_chunks(a.ctypes.data if a.size else None, a.size, fmt, None, 0, ctypes.byref(n))
    if rc not in (0, E_RANGE):
        _check(rc, "syncr_cdc_format_chunks")
    buf = ctypes.create_string_buffer(max(int(n.value), 1))
    _check(library().syncr_cdc_format_chunks(a.ctypes.data if a.size else None, a.size, fmt, buf, n.value,
                                             ctypes.byref(n)), "syncr_cdc_format_chunks")
    return buf.raw[: int(n.value)]


class ChunkCache:
    """Persistent chunk cache (syncr_cache_*), the reference's ChildCache
    (src/cache.rs:138-260): per key (file path) the file's mtime, size and
    ChunkInfo list; valid when mtime (cache.rs:175) and size match.  Bound to
    one set of chunking parameters (stored in the log header).  Host code:
    works without a GPU."""

    def __init__(self, path: Optional[str] = None, chunk_bits: int = CHUNK_BITS, max_chunk: int = MAX_CHUNK_SIZE,
                 read_cap: int = TOKIO_READ_CAP):
        h = _vp()
        self.params = Params(chunk_bits, 0, max_chunk, read_cap)
        _check(library().syncr_cache_open(os.fsencode(path) if path else None, ctypes.byref(self.params),
                                          ctypes.byref(h)), "syncr_cache_open")
        self._h = h

    @property
    def handle(self):
        return self._h

    def get(self, key: str, mtime: int, size: int) -> Optional[np.ndarray]:
        L = library()
        n = ctypes.c_uint64(0)
        k = os.fsencode(key)
        rc = L.syncr_cache_get(self._h, k, mtime, size, None, 0, ctypes.byref(n))
        if rc == E_NOENT:
            return None
        if rc == 0:                          # a hit with no chunks (an empty file)
            return np.zeros(0, CHUNK_INFO_DTYPE)
        if rc != E_RANGE:
            _check(rc, "syncr_cache_get")
        out = np.zeros(max(int(n.value), 1), CHUNK_INFO_DTYPE)
        _check(L.syncr_cache_get(self._h, k, mtime, size, out.ctypes.data, out.size, ctypes.byref(n)),
               "syncr_cache_get")
        return out[: int(n.value)]

    def put(self, key: str, mtime: int, size: int, chunks: np.ndarray) -> None:
        a = np.ascontiguousarray(chunks, dtype=CHUNK_INFO_DTYPE)
        _check(library().syncr_cache_put(self._h, os.fsencode(key), mtime, size, a.ctypes.data if a.size else None,
                                         a.size), "syncr_cache_put")

    def sync(self) -> None:
        _check(library().syncr_cache_sync(self._h), "syncr_cache_sync")

    def stats(self) -> dict:
        st = (ctypes.c_uint64 * 4)()
        _check(library().syncr_cache_stats(self._h, st), "syncr_cache_stats")
        return {"hits": st[0], "misses": st[1], "puts": st[2], "entries": st[3]}

    def close(self) -> None:
        if getattr(self, "_h", None):
            library().syncr_cache_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Ingest:
    """Batched ingest pipeline (syncr_ingest_*): the directory walk of
    traverse_and_stream (file_operations.rs:544-715) without its serial
    per-file await.  Files go into pinned staging batches; each sealed batch is
    chunked + hashed on the GPU while the next fills.  Results arrive in
    submission order as (tag, status, ChunkInfo structured array) through
    `on_file`, or are collected in `.results` when no callback is given.
    devices=[d0, d1, ...]: one sub-pipeline and worker thread per listed device
    (syncr_ingest_open_multi), files assigned whole to the least-loaded one."""

    def __init__(self, chunk_bits: int = CHUNK_BITS, max_chunk: int = MAX_CHUNK_SIZE,
                 read_cap: int = TOKIO_READ_CAP, device: int = 0, batch_bytes: int = 256 << 20,
                 depth: int = 3, copy_threads: int = 8, on_file=None, cache: Optional["ChunkCache"] = None,
                 devices: Optional[Sequence[int]] = None):
        L = library()
        self.params = Params(chunk_bits, 0, max_chunk, read_cap)
        self.results: list[tuple[int, int, np.ndarray]] = []
        self._user = on_file

        def cb(_ctx, tag, status, ptr, n):
            a = np.zeros(n, CHUNK_INFO_DTYPE)
            if n:
                ctypes.memmove(a.ctypes.data, ptr, n * CHUNK_INFO_DTYPE.itemsize)
            if self._user is not None:
                self._user(int(tag), int(status), a)
            else:
                self.results.append((int(tag), int(status), a))

        self._cb = _INGEST_CB(cb)           # keep alive for the handle's lifetime
        h = _vp()
        if devices is None:
            _check(L.syncr_ingest_open(device, ctypes.byref(self.params), batch_bytes, depth, copy_threads,
                                       self._cb, None, ctypes.byref(h)), "syncr_ingest_open")
            self.devices = [device]
        else:
            self.devices = [int(d) for d in devices]
            arr = (_i32 * len(self.devices))(*self.devices)
            _check(L.syncr_ingest_open_multi(arr, len(self.devices), ctypes.byref(self.params), batch_bytes, depth,
                                             copy_threads, self._cb, None, ctypes.byref(h)), "syncr_ingest_open_multi")
        self._h = h
        self._cache = cache                  # keep alive while attached
        if cache is not None:
            _check(L.syncr_ingest_set_cache(h, cache.handle), "syncr_ingest_set_cache")

    def submit(self, data, tag: int) -> None:
        a = _u8(data)
        _check(library().syncr_ingest_submit(self._h, a.ctypes.data if a.size else None, a.size, tag),
               "syncr_ingest_submit")

    def submit_file(self, path, tag: int) -> None:
        _check(library().syncr_ingest_submit_file(self._h, os.fsencode(path), tag), "syncr_ingest_submit_file")

    def reserve(self, n: int) -> np.ndarray:
        """Zero-copy: a writable view of n bytes of pinned staging; commit() after filling."""
        p = _vp()
        _check(library().syncr_ingest_reserve(self._h, n, ctypes.byref(p)), "syncr_ingest_reserve")
        if not n:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))

    def commit(self, tag: int) -> None:
        _check(library().syncr_ingest_commit(self._h, tag), "syncr_ingest_commit")

    def flush(self) -> None:
        _check(library().syncr_ingest_flush(self._h), "syncr_ingest_flush")

    def stats(self) -> dict:
        st = (ctypes.c_uint64 * 4)()
        _check(library().syncr_ingest_stats(self._h, st), "syncr_ingest_stats")
        hits = ctypes.c_uint64(0)
        _check(library().syncr_ingest_cache_hits(self._h, ctypes.byref(hits)), "syncr_ingest_cache_hits")
        return {"files": st[0], "bytes": st[1], "batches": st[2], "chunks": st[3], "cache_hits": hits.value}

    def set_read_fault(self, offset: int | None, err: int = 0) -> None:
        """Fault injection for tests of the read-error contract: later
        submit_file calls read only the bytes before `offset`; the read that
        would cross it fails with errno `err` (0: EOF there, a file that
        shrank). offset None turns it off."""
        off = 2**64 - 1 if offset is None else offset
        _check(library().syncr_ingest_set_read_fault(self._h, off, err), "syncr_ingest_set_read_fault")

    def timing(self) -> dict:
        """Host seconds per pipeline stage so far (syncr_ingest_timing)."""
        t = (ctypes.c_double * 5)()
        _check(library().syncr_ingest_timing(self._h, t, 5), "syncr_ingest_timing")
        return dict(zip(("copy", "read", "seal", "wait", "deliver"), (round(x, 6) for x in t)))

    def device_stats(self) -> list[dict]:
        """Per sub-pipeline: device, files, bytes, batches."""
        n = 4 * len(self.devices)
        st = (ctypes.c_uint64 * n)()
        _check(library().syncr_ingest_device_stats(self._h, st, n), "syncr_ingest_device_stats")
        return [{"device": st[4 * k], "files": st[4 * k + 1], "bytes": st[4 * k + 2], "batches": st[4 * k + 3]}
                for k in range(len(self.devices))]

    def close(self) -> None:
        if getattr(self, "_h", None):
            library().syncr_ingest_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _split(cuts: np.ndarray, counts: np.ndarray) -> list[np.ndarray]:
    out, o = [], 0
    for c in counts.tolist():
        out.append(cuts[o: o + int(c)])
        o += int(c)
    return out


_default: Optional[Chunker] = None


def _default_chunker() -> Chunker:
    global _default
    if _default is None:
        _default = Chunker()
    return _default


def compute_file_chunks(path, chunker: Optional[Chunker] = None, hashed: bool = True) -> list[ChunkInfo]:
    """compute_file_chunks (src/protocol/file_operations.rs:721-788): chunk one
    file with production semantics and hash every chunk (BLAKE3, :757), both on
    the GPU.  Like the reference, an unreadable file is logged and yields an
    empty list (:727-744); GPU errors raise."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError as e:
        log.warning("Cannot open file %s: %s", path, e)
        return []
    return (chunker or _default_chunker()).chunk_bytes(data, hashed=hashed)


def chunk_data(data, chunk_bits: int = 13, max_chunk: Optional[int] = None,
               chunker: Optional[Chunker] = None) -> list[tuple[int, int]]:
    """tests/chunking_test.rs:170-192: in-memory ideal semantics, (offset, size)
    pairs; defaults are that test's CHUNK_BITS=13, MAX=(1<<13)*16 (:7-8)."""
    if chunker is None:
        max_chunk = max_chunk or (1 << chunk_bits) * 16
        with Chunker(chunk_bits, max_chunk, 0) as c:
            return [(ci.offset, ci.size) for ci in c.chunk_bytes(data)]
    return [(ci.offset, ci.size) for ci in chunker.chunk_bytes(data)]
