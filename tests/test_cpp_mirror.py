"""The C++ host mirror (include/syncr_cdc.hpp) compiles against the C ABI on
the CPU, and its chunking_test mirror passes on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "chunking_test")


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
