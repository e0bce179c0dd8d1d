#!/usr/bin/env python3
"""Timeline of one resolve launch (development library, SYNCR_CDC_TRACE=1).

The resolve kernel stamps wall_clock64 (Tables::dbg, cdc_internal.h DBG_*):
the dense pass's waves (entry, end, and issue / landing / roll end / fix-up end of
the first tiles of 16 waves), the resolve kernel's block 0 start, the largest split file's walker (entry, after its split
setup, each block of 64 adopted records, walk end), every split worker's walk
(start, end) of records < DBG_NREC, and the copy launch's start.  Printed in us from
the resolve kernel's first wave.

    python tools/resolve_timeline.py --workload dense1 [VAR=VAL ...]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import syncr_amd  # noqa: E402

syncr_amd.use_dev_library()

DBG_RES_START, DBG_RES_END, DBG_W_ENTRY, DBG_W_SETUP, DBG_W_END, DBG_W_NBLK = 0, 1, 2, 3, 4, 5
DBG_W_BLK, DBG_COPY_START, DBG_COPY_END, DBG_REC, DBG_NREC = 8, 248, 249, 256, 1024
DBG_FW, DBG_NFW = DBG_REC + 2 * DBG_NREC, 1024
DBG_SCAN = DBG_FW + DBG_NFW
DBG_CW, DBG_NCW = DBG_SCAN + 4 * 4096 + 16 * 128, 4096      # split copy waves: end, start
DBG_DW, DBG_NDW = DBG_CW + 2 * DBG_NCW, 2048                   # dense-pass waves: entry, end | tiles << 56
DBG_DT, DBG_DT_W, DBG_DT_N = DBG_DW + 2 * DBG_NDW, 16, 16       # their first tiles: issue, landed, rolled, fixed
WORDS = DBG_DT + 4 * DBG_DT_W * DBG_DT_N


def dense_timeline(d):
    """The dense pass's waves, in us from its first wave's entry."""
    dw = d[DBG_DW:DBG_DW + 2 * DBG_NDW].reshape(-1, 2)
    live = (dw[:, 0] > 0) & (dw[:, 1] > 0)
    if not live.any():
        return
    mask = (1 << 56) - 1
    ent = dw[live, 0].astype(np.int64)
    end = (dw[live, 1] & np.uint64(mask)).astype(np.int64)
    ntl = (dw[live, 1] >> np.uint64(56)).astype(np.int64)
    t0 = ent.min()
    us = lambda v: (v - t0) / 100.0                                    # noqa: E731
    e, x = us(ent), us(end)
    print(f"  dense waves ({live.sum()}): entry p50 {np.median(e):.1f} max {e.max():.1f}; end p10 "
          f"{np.percentile(x, 10):.1f} p50 {np.median(x):.1f} p90 {np.percentile(x, 90):.1f} max {x.max():.1f}; "
          f"tiles per wave p50 {np.median(ntl):.0f} max {ntl.max()}")
    dt = d[DBG_DT:DBG_DT + 4 * DBG_DT_W * DBG_DT_N].reshape(DBG_DT_W, DBG_DT_N, 4).astype(np.int64)
    lat, roll, fix, gap = [], [], [], []
    for w in range(DBG_DT_W):
        for k in range(DBG_DT_N):
            iss, land, rl, fx = dt[w, k]
            if not (iss and land and rl and fx):
                continue
            lat.append((land - iss) / 100.0)
            roll.append((rl - land) / 100.0)
            fix.append((fx - rl) / 100.0)
            if k + 1 < DBG_DT_N and dt[w, k + 1, 1]:
                gap.append((dt[w, k + 1, 1] - fx) / 100.0)
    if lat:
        q = lambda v: f"p50 {np.median(v):.2f} p90 {np.percentile(v, 90):.2f} max {max(v):.2f}"   # noqa: E731
        print(f"  dense tiles ({len(lat)} of {DBG_DT_W} waves): issue->landed {q(lat)}; roll {q(roll)}; "
              f"fix-ups {q(fix)}; fix-ups end->next landed {q(gap) if gap else '-'}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("env", nargs="*")
    ap.add_argument("--workload", default="dense1")
    ap.add_argument("--launches", type=int, default=4)
    args = ap.parse_args()
    for kv in args.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    os.environ["SYNCR_CDC_TRACE"] = "1"
    if args.workload == "shard8":                   # BASELINE config 4's rank-0 batch at N = 8
        from benchlib import workloads as WL
        z = WL.zipf_sizes()
        sh = WL.lpt_shard(z, 8)[0]
        sizes, idx = z[sh], sh.astype(np.uint64)
    else:
        sizes, idx, _ = bench.workload(args.workload, 1)
    offs = np.zeros_like(sizes)
    offs[1:] = np.cumsum(sizes)[:-1]
    span = int(sizes.sum())
    c = syncr_amd.Chunker()
    buf = syncr_amd.DeviceBuffer(c, span)
    buf.gen_corpus(offs, sizes, indices=idx)
    if args.workload == "dense":
        from benchlib import legs
        legs.fill_dense(buf, offs, sizes, idx)
    elif args.workload == "dense1":
        buf.upload(np.resize(bench.periodic_pattern(), span))
    c.plan(offs, sizes, span)
    L = syncr_amd.library()
    L.syncr_cdc_dev_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    L.syncr_cdc_dev_trace.restype = ctypes.c_int32
    c.launch(buf.ptr)
    c.fetch()                               # the fetch turns the split hint on
    for n in range(args.launches):
        c.launch(buf.ptr)
        d = np.zeros(WORDS, np.uint64)
        assert L.syncr_cdc_dev_trace(c.handle, d.ctypes.data, WORDS) == 0
        t0 = int(d[DBG_RES_START])
        us = lambda v: (int(v) - t0) / 100.0 if v else None          # 100 MHz wall clock
        print(f"launch {n}: split {c.split_stats()}")
        print(f"  block 0: after zero_next {us(d[6])}, file loads {us(d[7])}")
        print(f"  walker entry {us(d[DBG_W_ENTRY])} setup {us(d[DBG_W_SETUP])} "
              f"end {us(d[DBG_W_END])}")
        nb = int(d[DBG_W_NBLK])
        blk = [(us(d[DBG_W_BLK + 2 * b]), us(d[DBG_W_BLK + 2 * b + 1])) for b in range(min(nb, 60))]
        print(f"  walker adoption blocks ({nb}): " + ", ".join(f"{a:.1f}-{b:.1f}" for a, b in blk[:24]))
        rec = d[DBG_REC:DBG_FW].reshape(-1, 2)
        have = rec[:, 0] > 0
        if have.any():
            st = np.array([us(v) for v in rec[have, 0]])
            en = np.array([us(v) for v in rec[have, 1] if v] or [0.0])
            dur = en[:st.size] - st[:en.size]
            print(f"  worker walks ({have.sum()}): start min {st.min():.1f} med {np.median(st):.1f} "
                  f"max {st.max():.1f}; end max {en.max():.1f}; duration med {np.median(dur):.1f} max {dur.max():.1f}")
        print(f"  copy start {us(d[DBG_COPY_START])}")
        cw = d[DBG_CW:DBG_CW + 2 * DBG_NCW].reshape(-1, 2)
        live = cw[:, 0] > 0
        if live.any():
            ce = np.array([us(v) for v in cw[live, 0]])
            cs = np.array([us(v) for v in cw[live, 1]])
            dur = ce - cs
            print(f"  copy wave ends ({live.sum()}): p50 {np.percentile(ce, 50):.1f} p90 {np.percentile(ce, 90):.1f} "
                  f"max {ce.max():.1f}; starts p50 {np.percentile(cs, 50):.1f} p90 {np.percentile(cs, 90):.1f} "
                  f"max {cs.max():.1f}; durations p50 {np.percentile(dur, 50):.1f} p90 {np.percentile(dur, 90):.1f} "
                  f"max {dur.max():.1f}; waves by wid/1024: "
                  + ", ".join(f"{np.median(dur[(np.nonzero(live)[0] // 1024) == b]):.1f}" for b in range(4)))
        dense_timeline(d)
        fw = d[DBG_FW:DBG_FW + DBG_NFW]
        ends = sorted(((us(v), k) for k, v in enumerate(fw) if v), reverse=True)[:6]
        order = np.argsort(-sizes.astype(np.int64), kind="stable")
        print("  latest file walkers (end us, order index, size KiB, corpus index): " +
              ", ".join(f"{e:.1f}/{k}/{int(sizes[order[k]]) >> 10}/{int(idx[order[k]])}" for e, k in ends))
        allw = np.array([us(v) for v in fw if v])
        if allw.size:
            print(f"  file walker ends ({allw.size}): p50 {np.percentile(allw, 50):.1f} p90 {np.percentile(allw, 90):.1f} "
                  f"p99 {np.percentile(allw, 99):.1f} max {allw.max():.1f}; resolve end {us(d[DBG_RES_END])}")
    buf.free()


if __name__ == "__main__":
    main()
