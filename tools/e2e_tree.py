#!/usr/bin/env python3
"""Write the first N zipf10k files (the bench's corpus bytes, generated on the
host by the xorshift rule) as a directory tree for benchlib/e2e_driver.cpp, so
one driver mode can be run alone (e.g. under rocprofv3).

    python tools/e2e_tree.py ROOT [--files N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from benchlib import workloads as WL  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--files", type=int, default=1000)
    a = ap.parse_args()
    sizes = WL.zipf_sizes()[: a.files]
    idx = np.arange(sizes.size, dtype=np.uint64)
    host, offs = O.corpus_fill_threads(sizes, indices=idx)
    for j in range(sizes.size):
        d = os.path.join(a.root, f"d{j // 100:03d}")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"f{j:07d}.bin"), "wb") as f:
            f.write(memoryview(host[int(offs[j]): int(offs[j] + sizes[j])]))
    print(f"{sizes.size} files, {int(sizes.sum())} bytes under {a.root}")


if __name__ == "__main__":
    main()
