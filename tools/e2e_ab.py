#!/usr/bin/env python3
"""Same-box A/B of the end-to-end legs: benchlib/e2e_driver.cpp run against
two (or more) builds of the product library, interleaved, over one tree of
the first N zipf10k files.  The driver finds libsyncr_cdc.so through its
RUNPATH, so LD_LIBRARY_PATH=<dir> swaps the library under the same binary
(the C ABI is unchanged between the builds compared).

    python tools/e2e_ab.py --libs syncr_amd,build/ab_pre/syncr_amd \
        [--modes files,mem,zero_copy,walk] [--rounds 3] [--files 10000]

Prints one JSON line per (round, lib, mode) and a per-lib median summary.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from benchlib import e2e as E  # noqa: E402
from benchlib import workloads as WL  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--modes", default="files,mem,zero_copy,walk")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--files", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    libs = [os.path.join(ROOT, x) for x in a.libs.split(",")]
    binary = E.driver()
    sizes = WL.zipf_sizes()[: a.files]
    idx = np.arange(sizes.size, dtype=np.uint64)
    host, offs = O.corpus_fill_threads(sizes, indices=idx)
    root, nfiles = E.write_tree(host, offs, sizes, idx)
    del host
    res = {}
    try:
        for r in range(a.rounds):
            for lib in libs:
                for mode in a.modes.split(","):
                    env = dict(os.environ, LD_LIBRARY_PATH=lib)
                    t0 = time.perf_counter()
                    p = subprocess.run([binary, mode, root, "/dev/null", "--reps", str(a.reps)], env=env,
                                       capture_output=True, text=True, timeout=300)
                    if p.returncode:
                        print(json.dumps({"lib": lib, "mode": mode, "error": p.stderr[-400:]}), flush=True)
                        sys.exit(1)
                    d = json.loads(p.stdout.strip().splitlines()[-1])
                    v = d["bytes"] / min(d["pass_seconds"]) / 2**30
                    res.setdefault((lib, mode), []).append(v)
                    print(json.dumps({"round": r, "lib": os.path.relpath(lib, ROOT), "mode": mode,
                                      "gib_s": round(v, 3), "pass_seconds": d["pass_seconds"],
                                      "stage": d["host_stage_seconds"], "wall": round(time.perf_counter() - t0, 1)}),
                          flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    print(json.dumps({"summary": {f"{os.path.relpath(l, ROOT)}:{m}": round(float(np.median(v)), 3)
                                  for (l, m), v in res.items()}, "files": nfiles}))


if __name__ == "__main__":
    main()
