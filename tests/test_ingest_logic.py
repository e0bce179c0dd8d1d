"""Host logic of the (multi-device) ingest pipeline, on the CPU: device
assignment (online LPT by file size), in-order delivery across worker threads,
and the read-error rule of compute_file_chunks (file_operations.rs:776-782)
checked against the oracle's literal loop with a failing reader.  Compiles
tests/cpp/ingest_logic_test.cpp with g++ against syncr_amd/csrc/ingest_logic.h."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ingest_logic_cpp():
    from oracle import oracle as O
    O.build()
    odir = os.path.join(ROOT, "oracle")
    binary = os.path.join(ROOT, "build", "ingest_logic_test")
    os.makedirs(os.path.dirname(binary), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "syncr_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "ingest_logic_test.cpp"), os.path.join(odir, "liborc_bup.so"),
                    f"-Wl,-rpath,{odir}", "-lpthread", "-o", binary], check=True)
    r = subprocess.run([binary], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
