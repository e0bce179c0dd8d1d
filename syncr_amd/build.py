"""Build libsyncr_cdc.so (HIP kernels + C ABI) in-tree with hipcc for gfx950."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libsyncr_cdc.so")
# development library: the same sources with -DSYNCR_CDC_DEV (scan variants,
# MFMA scan, timing-only ablations chosen by environment variables); used by
# tools/ only, never by the product path or the parity tests
DEV_LIB = os.path.join(PKG, "libsyncr_cdc_dev.so")
SOURCES = [os.path.join(CSRC, "cdc_kernels.hip"), os.path.join(CSRC, "b3_kernels.hip"),
           os.path.join(CSRC, "cdc_api.cpp"), os.path.join(CSRC, "ingest.cpp"),
           os.path.join(CSRC, "cache.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, "cdc_internal.h"), os.path.join(CSRC, "lds_dma.h"),
                  os.path.join(CSRC, "ingest_logic.h"), os.path.join(ROOT, "include", "syncr_cdc.h")]
# development-only kernels and launchers, #included under SYNCR_CDC_DEV (the product build never reads them)
DEV_DEPS = [os.path.join(CSRC, "dev", f) for f in ("scan_mfma.inc", "dense_generic.inc", "scan_launch_dev.inc")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SYNCR_CDC_ARCH", "gfx950")


def needs_build(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in DEPS + (DEV_DEPS if lib == DEV_LIB else []))


def build(force: bool = False, verbose: bool = False, dev: bool = False) -> str:
    lib = DEV_LIB if dev else LIB
    if not force and not needs_build(lib):
        return lib
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"),
           "-o", lib + ".tmp", *SOURCES]
    if dev:
        cmd[1:1] = ["-DSYNCR_CDC_DEV", "-mllvm", "-amdgpu-mfma-vgpr-form"]   # MFMA scan: results in VGPRs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, dev="--dev" in sys.argv))
