"""The C++ host mirror (include/syncr_cdc.hpp) compiles against the C ABI on
the CPU, and its chunking_test mirror passes on the GPU; the Rust shim's call
sequence (rust/src/chunking_gpu.rs), restated in C++ against the oracle,
compiles here and passes on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "chunking_test")
SHIM_BIN = os.path.join(ROOT, "build", "shim_sequence_test")


def build_mirror():
    from syncr_amd import build as B
    B.build()
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    pkg = os.path.join(ROOT, "syncr_amd")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "chunking_test.cpp"),
                    os.path.join(pkg, "libsyncr_cdc.so"), f"-Wl,-rpath,{pkg}", "-o", BIN], check=True)
    return BIN


def test_cpp_mirror_compiles():
    assert os.path.exists(build_mirror())


@pytest.mark.gpu
def test_cpp_mirror_runs(tmp_path):
    binary = build_mirror()
    r = subprocess.run([binary], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


def build_shim_test():
    """tests/cpp/shim_sequence_test.cpp against the product library and the
    oracle (the checker)."""
    from syncr_amd import build as B
    from oracle import oracle as O
    B.build()
    O.lib()                                          # builds oracle/liborc_bup.so if stale
    os.makedirs(os.path.dirname(SHIM_BIN), exist_ok=True)
    pkg, orc = os.path.join(ROOT, "syncr_amd"), os.path.join(ROOT, "oracle")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_sequence_test.cpp"),
                    os.path.join(pkg, "libsyncr_cdc.so"), os.path.join(orc, "liborc_bup.so"),
                    f"-Wl,-rpath,{pkg}", f"-Wl,-rpath,{orc}", "-o", SHIM_BIN], check=True)
    return SHIM_BIN


def test_shim_sequence_compiles():
    assert os.path.exists(build_shim_test())


@pytest.mark.gpu
def test_shim_sequence_runs(tmp_path):
    """The Rust shim's exact sequence through the C ABI: ingest depth 1,
    submit_file -> flush -> one callback per file -> close (random, oversized,
    empty, b"small", periodic, constant, missing, a directory; twice), and
    chunk_host_hashed with the ERANGE retry; every ChunkInfo list vs the oracle."""
    binary = build_shim_test()
    r = subprocess.run([binary], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "all checks passed" in r.stdout


WALK_BIN = os.path.join(ROOT, "build", "walk_sequence_test")


def build_walk_test():
    """tests/cpp/walk_sequence_test.cpp against the product library and the
    oracle (the checker)."""
    from syncr_amd import build as B
    from oracle import oracle as O
    B.build()
    O.lib()
    os.makedirs(os.path.dirname(WALK_BIN), exist_ok=True)
    pkg, orc = os.path.join(ROOT, "syncr_amd"), os.path.join(ROOT, "oracle")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "walk_sequence_test.cpp"),
                    os.path.join(pkg, "libsyncr_cdc.so"), os.path.join(orc, "liborc_bup.so"),
                    f"-Wl,-rpath,{pkg}", f"-Wl,-rpath,{orc}", "-o", WALK_BIN], check=True)
    return WALK_BIN


def test_walk_sequence_compiles():
    assert os.path.exists(build_walk_test())


@pytest.mark.gpu
def test_walk_sequence_runs(tmp_path):
    """The batched walk (GpuWalk: the traverse_and_stream patch) through the C
    ABI over a nested tree -- random, empty, b"small", periodic, constant,
    oversized, 300 small files, a vanishing file, an unreadable file, a symlink,
    an empty directory -- on one device with small batches (twice), on devices
    {0, 0} and with the shim's defaults: the entry sequence equals the
    reference walk's and every file's status and ChunkInfo list the oracle's."""
    binary = build_walk_test()
    r = subprocess.run([binary], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "all checks passed" in r.stdout


def reference_walk_order(base):
    """traverse_and_stream's order (src/protocol/file_operations.rs:551-703),
    restated: a stack of directories, each read in readdir order (os.listdir),
    lstat per entry, files / symlinks / directories emitted, directories pushed
    when met."""
    out, stack = [], [base]
    while stack:
        d = stack.pop()
        try:
            names = os.listdir(d)
        except OSError:
            continue
        for n in names:
            p = os.path.join(d, n)
            try:
                st = os.lstat(p)
            except OSError:
                continue
            import stat as S
            rel = os.path.relpath(p, base)
            if S.S_ISREG(st.st_mode):
                out.append((rel, "F", st.st_size, ""))
            elif S.S_ISLNK(st.st_mode):
                out.append((rel, "S", 0, os.readlink(p)))
            elif S.S_ISDIR(st.st_mode):
                out.append((rel, "D", 0, ""))
                stack.append(p)
    return out


def test_walk_tree_order_matches_reference(tmp_path):
    """syncr::walk_tree (include/syncr_cdc.hpp, used by GpuWalk's C++ mirror and
    the end-to-end driver) emits the reference walk's sequence; no device."""
    from benchlib import e2e as E
    binary = E.driver()
    base = tmp_path / "tree"
    for d in ("a", "a/b", "a/b/c", "e", "z"):
        (base / d).mkdir(parents=True)
    for i, f in enumerate(("x", "a/y", "a/b/z", "a/b/c/w", "e/v", "z/u1", "z/u2", "q")):
        (base / f).write_bytes(b"k" * (i * 7))
    os.symlink("../a", base / "e" / "up")
    os.mkfifo(base / "fifo")                       # neither file, directory nor symlink: skipped
    r = subprocess.run([binary, "list", str(base), "-"], capture_output=True, text=True, timeout=60, check=True)
    got = [tuple(l.split("\t")) for l in r.stdout.splitlines()]
    got = [(a, b, int(c), d) for a, b, c, d in got]
    assert got == reference_walk_order(str(base))
