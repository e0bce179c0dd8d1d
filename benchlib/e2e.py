"""End-to-end legs of bench.py driven from C++ (benchlib/e2e_driver.cpp): the
zipf10k corpus written to a directory tree on local disk, then chunked + hashed
by the product library through the calls syncr's Rust host makes, with no
Python per file.  Every file's ChunkInfo list is checked
against the golden digests (tests/golden/zipf10k_digests.npz).

    shim_per_file   the round-5 integration: the reference's walk awaiting each
                    file on a depth-1 pipeline (submit_file -> flush)
    shim_walk       the batched walk (GpuWalk + the traverse_and_stream patch)
    ingest_files    the file list through submit_file, one flush
    ingest          files in host memory through submit (library copies)
    ingest_zero_copy  the same bytes through reserve / caller fill / commit
"""
from __future__ import annotations

import json
import os
import re
import shutil
import subprocess
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from benchlib import golden as G

ROOT = G.ROOT
SRC = os.path.join(ROOT, "benchlib", "e2e_driver.cpp")
BIN = os.path.join(ROOT, "build", "e2e_driver")
FILES_PER_DIR = 100
_NAME = re.compile(r"f(\d+)\.bin$")


def driver() -> str:
    """build/e2e_driver (g++ against the product library), rebuilt when stale."""
    from syncr_amd import build as B
    lib = B.build()
    deps = [SRC, os.path.join(ROOT, "include", "syncr_cdc.hpp"), os.path.join(ROOT, "include", "syncr_cdc.h"), lib]
    if not os.path.exists(BIN) or any(os.path.getmtime(p) > os.path.getmtime(BIN) for p in deps):
        os.makedirs(os.path.dirname(BIN), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-I",
                        os.path.join(ROOT, "include"), SRC, lib, "-Wl,-rpath,$ORIGIN/../syncr_amd",
                        "-o", BIN + ".tmp"], check=True)
        os.replace(BIN + ".tmp", BIN)
    return BIN


def write_tree(host: np.ndarray, offs, lens, idx, budget_bytes: int | None = None) -> tuple[str, int]:
    """The files as a directory tree: <root>/dNNN/fIIIIIII.bin (100 files per
    directory, I = corpus index), written and fsync'ed (clean page cache, no
    writeback under the timed passes).  Files are taken in corpus order while
    they fit in `budget_bytes` (None: the free space of the temp file system
    minus 2 GiB).  Returns (root, files written)."""
    root = tempfile.mkdtemp(prefix="syncr_e2e_")
    if budget_bytes is None:
        budget_bytes = shutil.disk_usage(root).free - (2 << 30)
    take, tot = [], 0
    for j in range(lens.size):
        if tot + int(lens[j]) > budget_bytes:
            break
        take.append(j)
        tot += int(lens[j])

    def one(j):
        d = os.path.join(root, f"d{j // FILES_PER_DIR:03d}")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"f{int(idx[j]):07d}.bin"), "wb") as f:
            f.write(memoryview(host[int(offs[j]): int(offs[j] + lens[j])]))
            f.flush()
            os.fsync(f.fileno())

    with ThreadPoolExecutor(16) as ex:
        list(ex.map(one, take))
    return root, len(take)


def read_results(path: str) -> list[tuple[str, int, np.ndarray]]:
    import syncr_amd
    out = []
    raw = open(path, "rb").read()
    p = 0
    while p < len(raw):
        (pl,) = np.frombuffer(raw, np.uint32, 1, p)
        p += 4
        name = raw[p:p + int(pl)].decode()
        p += int(pl)
        st, n = np.frombuffer(raw, np.int32, 1, p)[0], np.frombuffer(raw, np.uint32, 1, p + 4)[0]
        p += 8
        a = np.frombuffer(raw, syncr_amd.CHUNK_INFO_DTYPE, int(n), p).copy()
        p += int(n) * syncr_amd.CHUNK_INFO_DTYPE.itemsize
        out.append((name, int(st), a))
    return out


def run(mode: str, root: str, device: int = 0, reps: int = 2, timeout: int = 300) -> dict:
    """One driver run: its JSON line + parity of every delivered file."""
    binary = driver()
    fd, res_path = tempfile.mkstemp(prefix=f"syncr_e2e_{mode}_", suffix=".bin")
    os.close(fd)
    try:
        t0 = time.perf_counter()
        r = subprocess.run([binary, mode, root, res_path, "--reps", str(reps), "--device", str(device)],
                           capture_output=True, text=True, timeout=timeout)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            return {"error": f"e2e_driver {mode} rc={r.returncode}: {r.stderr[-800:]}"}
        out = json.loads(r.stdout.strip().splitlines()[-1])
        res = read_results(res_path)
    finally:
        os.unlink(res_path)
    rows = np.array([int(_NAME.search(n).group(1)) for n, _, _ in res], np.int64)
    out["parity"] = G.check_files("zipf10k", [a for _, _, a in res], rows, hashed=True)
    out["value"] = round(out["bytes"] / out["seconds"] / 2**30, 3) if out["seconds"] > 0 else None
    out["unit"] = "GiB/s"
    out["driver_wall_seconds"] = round(wall, 2)
    return out


PATHS = {
    "shim_per_file": "C++ caller (benchlib/e2e_driver.cpp per_file): the reference's walk (traverse_and_stream order) "
                     "awaiting each file on ONE pooled depth-1 pipeline (64 MiB batch, 4 threads), "
                     "submit_file -> flush -> one callback per file: what compute_file_chunks_gpu does today",
    "shim_walk": "C++ caller (e2e_driver walk): the batched walk, every file submitted to one pipeline (256 MiB "
                 "batches, depth 3, 16 threads) as the walk meets it, entries sent in walk order as results return "
                 "(GpuWalk, the traverse_and_stream patch in integration/file_operations.diff)",
    "ingest_files": "C++ caller (e2e_driver files): the tree's file list through syncr_ingest_submit_file (open + "
                    "fstat on the caller, pread into pinned staging on 16 pool threads), one flush",
    "ingest": "C++ caller (e2e_driver mem): every file first read into ordinary host memory (untimed), then "
              "syncr_ingest_submit per file (the library copies into pinned staging), one flush",
    "ingest_zero_copy": "C++ caller (e2e_driver zero_copy): the same host bytes through syncr_ingest_reserve -> the "
                        "caller's own copy into pinned staging (16 threads above 4 MiB) -> syncr_ingest_commit",
}
MODES = {"shim_per_file": "per_file", "shim_walk": "walk", "ingest_files": "files", "ingest": "mem",
         "ingest_zero_copy": "zero_copy"}


def legs(host: np.ndarray, offs, lens, idx, device: int, names=tuple(MODES)) -> dict:
    """Every end-to-end leg over one tree of the corpus's files."""
    t = time.perf_counter()
    root, nfiles = write_tree(host, offs, lens, idx)
    write_s = time.perf_counter() - t
    out = {}
    try:
        for name in names:
            r = run(MODES[name], root, device, reps=2 if name == "shim_per_file" else 3)
            r["path"] = PATHS[name]
            r["tree"] = (f"{nfiles} zipf10k files in {(nfiles + FILES_PER_DIR - 1) // FILES_PER_DIR} directories "
                         f"on local disk, written and fsync'ed before the passes (page cache, clean); "
                         f"written in {write_s:.1f} s")
            out[name] = r
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return out
