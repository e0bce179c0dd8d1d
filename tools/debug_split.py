#!/usr/bin/env python3
"""Debug: the test_split_walks configuration on the development library with
per-attempt fetch diagnostics (SYNCR_CDC_DEBUG_FETCH=1), twice per flag."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["SYNCR_CDC_DEBUG_FETCH"] = "1"
import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402

syncr_amd.use_dev_library()
M = 1 << 20
bits, mx, cap = [int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (8, 4096, 3000))]
rng = np.random.default_rng(bits * 7919 + cap)
files = []
lo, hi = (34 * M, 44 * M) if bits == 10 else (5 * M, 14 * M)
for k in range(3 if bits == 10 else 4):
    n = int(rng.integers(lo, hi))
    f = rng.integers(0, 256, n, dtype=np.uint8)
    f[n // 3: n // 3 + 200000] = 9
    files.append(f)
files.append(rng.integers(0, 256, 3 * M, dtype=np.uint8))
lens = np.array([f.size for f in files], np.uint64)
offs = np.zeros_like(lens)
offs[1:] = np.cumsum(lens + 48)[:-1]
span = int(offs[-1] + lens[-1]) + 16
data = np.zeros(span, np.uint8)
for o, f in zip(offs.tolist(), files):
    data[o:o + f.size] = f
want = [(O.chunk_production_window(data[o:o + n], bits, mx, cap) if cap else O.chunk_ideal(data[o:o + n], bits, mx)).tolist()
        for o, n in zip(offs.tolist(), lens.tolist())]
for flags in (0, syncr_amd.FLAG_RESOLVE_NOSPLIT, 0):
    for rep in range(2):
        print(f"--- flags {flags} rep {rep}", flush=True)
        try:
            with syncr_amd.Chunker(bits, mx, cap, flags=flags) as ch:
                res = ch.batch_arrays(data, offs, lens)
            for i in range(len(files)):
                e = (res[i]["offset"].astype(np.int64) + res[i]["len"].astype(np.int64)).tolist()
                print(f"file {i}: {len(e)} cuts, oracle {len(want[i])}, equal {e == want[i]}", flush=True)
        except syncr_amd.SyncrCdcError as ex:
            print("error", ex, flush=True)
