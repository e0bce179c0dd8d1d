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
