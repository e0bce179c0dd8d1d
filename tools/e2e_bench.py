#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) chunking rate: pinned host bytes -> H2D ->
scan/resolve -> cuts D2H, on the zipf10k corpus.

  serial:    one H2D of the whole corpus, one launch, one fetch
  pipelined: the file list split into P parts on P handles/streams; part k's
             H2D overlaps part k-1's kernels (copy engine || compute)

The corpus bytes are generated on the device and copied once to pinned host
memory (so host and device hold identical bytes); the timed region starts with
the bytes in pinned host memory and ends with all cuts in host memory.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402
from syncr_amd import _check, library  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    L = library()
    sizes, idx, _ = bench.workload("zipf10k", 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    ch = syncr_amd.Chunker()
    dev = syncr_amd.DeviceBuffer(ch, span)
    dev.gen_corpus(offs, sizes, indices=idx)
    hp = ctypes.c_void_p()
    _check(L.syncr_cdc_host_alloc_pinned(ch.handle, span, ctypes.byref(hp)), "host_alloc_pinned")
    _check(L.syncr_cdc_memcpy_d2h(ch.handle, hp.value, dev.ptr, span, None), "d2h")
    ch.synchronize()

    # ---- serial: H2D everything, launch, fetch ----
    ch.plan(offs, sizes, span)
    ser = []
    for _ in range(args.reps):
        ch.synchronize()
        t0 = time.perf_counter()
        _check(L.syncr_cdc_memcpy_h2d(ch.handle, dev.ptr, hp.value, span, None), "h2d")
        ch.launch(dev.ptr)
        cuts = ch.fetch()
        ser.append(time.perf_counter() - t0)
    ncuts = sum(c.size for c in cuts)

    # ---- pipelined: P contiguous file ranges on P handles / streams ----
    P = args.parts
    bounds = np.searchsorted(np.cumsum(sizes), np.linspace(0, span, P + 1)[1:-1])
    parts = np.split(np.arange(sizes.size), bounds + 1)
    hs = []
    for part in parts:
        if not part.size:
            continue
        o0 = int(offs[part[0]]) & ~15            # launch needs a 16-byte aligned base
        o1 = int(offs[part[-1]] + sizes[part[-1]])
        h = syncr_amd.Chunker()
        h.plan(offs[part] - np.uint64(o0), sizes[part], o1 - o0)
        hs.append((h, o0, o1))
    pip = []
    for _ in range(args.reps):
        for h, _, _ in hs:
            h.synchronize()
        t0 = time.perf_counter()
        for h, o0, o1 in hs:                      # copy and launch on the part's own stream
            s = h.stream
            _check(L.syncr_cdc_memcpy_h2d(h.handle, dev.ptr + o0, hp.value + o0, o1 - o0, s), "h2d")
            h.launch(dev.ptr + o0, s)
        tot = 0
        for h, _, _ in hs:
            tot += sum(c.size for c in h.fetch())
        pip.append(time.perf_counter() - t0)
    assert tot == ncuts, (tot, ncuts)
    out = {
        "workload": "zipf10k", "bytes": span, "cuts": ncuts,
        "serial_s": min(ser), "serial_GiBps": span / min(ser) / 2**30,
        "pipelined_parts": len(hs), "pipelined_s": min(pip), "pipelined_GiBps": span / min(pip) / 2**30,
        "h2d_note": "pinned host memory, hipMemcpyAsync; includes plan-free launches and cut D2H",
    }
    print(json.dumps(out))
    for h, _, _ in hs:
        h.close()
    L.syncr_cdc_host_free_pinned(ch.handle, hp.value)
    dev.free()


if __name__ == "__main__":
    main()
