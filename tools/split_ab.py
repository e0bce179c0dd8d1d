#!/usr/bin/env python3
"""One batch as two concurrent sub-batches (development A/B, config 4's shards).

A step is one batch, waited for before the next step (no overlap between
steps).  `one`: the batch as one launch.  `split<f>`: its files split into A
(the largest files, about 1 - f of the bytes: the stream-tile scan) and B (the
rest: a small batch, the CU-schedule scan), two handles, A launched then B on
another stream; the scans of different handles are not ordered, so B's waves
take the CUs A's last stream tiles free.

    python tools/split_ab.py [--fracs 0.1,0.2,0.3] [--steps 20] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from benchlib import golden as G  # noqa: E402
from benchlib import workloads as WL  # noqa: E402

HBM = 8000.0


def timed(groups, steps):
    """groups: list of (handle, buffer); each step launches every group and waits."""
    for _ in range(3):
        for h, b in groups:
            h.launch(b.ptr)
        for h, _ in groups:
            h.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for h, b in groups:
            h.launch(b.ptr)
        for h, _ in groups:
            h.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fracs", default="0.1,0.2,0.3")
    ap.add_argument("--shards", default="0,3,6")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--b-ablate", default="", help="dev library: SYNCR_CDC_ABLATE for B's handle (8: the "
                    "one-wave dynamic-group tile scan instead of the CU schedule)")
    a = ap.parse_args()
    if a.b_ablate:
        syncr_amd.use_dev_library()
    sizes = WL.zipf_sizes()
    shards = WL.lpt_shard(sizes, 8)
    fracs = [float(x) for x in a.fracs.split(",")]
    for r in [int(x) for x in a.shards.split(",")]:
        sh = shards[r]
        order = sh[np.argsort(sizes[sh], kind="stable")]          # smallest first
        total = int(sizes[sh].sum())
        made = {}

        def batch(idx, ablate=""):
            lens = sizes[idx]
            offs = WL.offsets_of(lens)
            span = int(lens.sum())
            if ablate:
                os.environ["SYNCR_CDC_ABLATE"] = ablate
            try:
                h = syncr_amd.Chunker()
            finally:
                os.environ.pop("SYNCR_CDC_ABLATE", None)
            b = syncr_amd.DeviceBuffer(h, max(span, 16))
            b.gen_corpus(offs, lens, indices=idx.astype(np.uint64))
            h.plan(offs, lens, span)
            h.launch(b.ptr)
            h.fetch()
            return (h, b, idx)

        made["one"] = [batch(sh)]
        for f in fracs:
            cum = np.cumsum(sizes[order])
            k = int(np.searchsorted(cum, f * total))
            made[f"split{f}"] = [batch(order[k:]), batch(order[:k], a.b_ablate)]
        ms = {m: [] for m in made}
        for _ in range(a.rounds):
            for m, grp in made.items():
                ms[m].append(timed([(h, b) for h, b, _ in grp], a.steps) * 1e3)
        mism = 0
        for grp in made.values():
            for h, b, idx in grp:
                mism += G.check_files("zipf10k", h.fetch(), idx.astype(np.int64))["mismatches"]
                b.free()
                h.close()
        row = {m: round(float(np.median(v)), 4) for m, v in ms.items()}
        row.update({f"{m}_frac": round(total / (v / 1e3) / 1e9 / HBM, 4) for m, v in list(row.items())})
        row["mismatches"] = mism
        print(json.dumps({f"shard{r}": row}), flush=True)


if __name__ == "__main__":
    main()
