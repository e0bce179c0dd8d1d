#!/usr/bin/env python3
"""Where a scan launch's time goes (development library, SYNCR_CDC_TRACE=1).

The dev scan kernel stamps wall_clock64 (100 MHz) per wave: entry, first tile
landed, exit, tiles rolled (cdc_internal.h DBG_SCAN), and every tile's landing
for the first DBG_TILE_W waves (DBG_TILE).  Printed per workload, for the last
of W+K back-to-back launches (and for the first launch after a host gap):

  entry spread     last wave's entry after the first (dispatch ramp)
  first land       a wave's first tile landing after its entry (DMA ramp)
  ends             wave exits (min / p10 / median / p90 / max) from the first entry
  tile             per-tile time of the sampled waves (steady roll + wait)
  resolve start    the resolve kernel's first stamp after the last scan wave's exit
                   (dense pass, compaction, fix-ups and the launch gaps between)

    python tools/scan_timeline.py [--workload uniform1k|shard8|zipf10k|dense1] [--shard R]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import syncr_amd  # noqa: E402
from benchlib import workloads as WL  # noqa: E402

syncr_amd.use_dev_library()

DBG_REC, DBG_NREC, DBG_NFW = 256, 1024, 1024
DBG_FW = DBG_REC + 2 * DBG_NREC
DBG_SCAN, DBG_SCAN_N = DBG_FW + DBG_NFW, 4096
DBG_TILE, DBG_TILE_W, DBG_TILE_N = DBG_SCAN + 4 * DBG_SCAN_N, 16, 128
WORDS = DBG_TILE + DBG_TILE_W * DBG_TILE_N


def table(name, shard):
    sizes = WL.zipf_sizes()
    if name == "uniform1k":
        lens = np.full(1024, 1 << 20, np.uint64)
        return lens, np.arange(1024, dtype=np.uint64)
    if name == "dense1":
        return np.full(1, 128 << 20, np.uint64), np.arange(1, dtype=np.uint64)
    if name == "shard8":
        sh = WL.lpt_shard(sizes, 8)[shard]
        return sizes[sh], sh.astype(np.uint64)
    return sizes, np.arange(sizes.size, dtype=np.uint64)


def summarize(d, grid):
    sc = d[DBG_SCAN:DBG_SCAN + 4 * DBG_SCAN_N].reshape(-1, 4)[:grid].astype(np.int64)
    have = sc[:, 0] > 0
    sc = sc[have]
    meta = sc[:, 3].copy()
    sc[:, 3] = meta & 0x0FFFFFFF                                    # tiles rolled
    xcc = (meta >> 28) & 0xF
    hw = (meta >> 32) & 0xFFFFFFFF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    t0 = sc[:, 0].min()
    us = lambda v: (v - t0) / 100.0                                  # noqa: E731
    ends = us(sc[:, 2])
    tiles = d[DBG_TILE:DBG_TILE + DBG_TILE_W * DBG_TILE_N].reshape(DBG_TILE_W, DBG_TILE_N).astype(np.uint64)
    per_tile = []
    seg_by_g = {}                                   # stream-tile scan: landing-to-landing time by segment index
    wait_by_g, work_by_g = {}, {}                   # stream tiles: wait at the landing / work before it
    for w in range(DBG_TILE_W):
        raw = tiles[w][tiles[w] > 0]
        arr = (raw >> np.uint64(55)) & np.uint64(1)
        g = (raw >> np.uint64(56)).astype(np.int64)
        t = (raw & np.uint64((1 << 55) - 1)).astype(np.int64)
        if arr.any():                               # stream-tile kernel: (arrive, landed) pairs
            land = np.nonzero(arr == 0)[0]
            for j, k in enumerate(land):
                if k > 0 and arr[k - 1]:
                    wait_by_g.setdefault(int(g[k]), []).append(float(t[k] - t[k - 1]) / 100.0)
                    if j > 0:
                        work_by_g.setdefault(int(g[k]), []).append(float(t[k - 1] - t[land[j - 1]]) / 100.0)
            g, t = g[land], t[land]
        if t.size > 2:
            dt = np.diff(t)
            per_tile.extend(dt.tolist())
            for k in range(1, t.size):
                seg_by_g.setdefault(int(g[k]), []).append(float(dt[k - 1]) / 100.0)
    per_tile = np.array(per_tile, np.float64) / 100.0
    res = int(d[0])
    out = {
        "waves": int(have.sum()),
        "entry_spread_us": round(float(us(sc[:, 0]).max()), 2),
        "first_land_us": {"median": round(float(np.median((sc[:, 1] - sc[:, 0]) / 100.0)), 2),
                          "max": round(float(((sc[:, 1] - sc[:, 0]) / 100.0).max()), 2)},
        "ends_us": {q: round(float(np.percentile(ends, p)), 2) for q, p in
                    (("min", 0), ("p10", 10), ("median", 50), ("p90", 90), ("max", 100))},
        "tiles_per_wave": {"min": int(sc[:, 3].min()), "max": int(sc[:, 3].max()),
                           "mean": round(float(sc[:, 3].mean()), 2)},
        "tile_us": ({"median": round(float(np.median(per_tile)), 3), "p10": round(float(np.percentile(per_tile, 10)), 3),
                     "p90": round(float(np.percentile(per_tile, 90)), 3), "first": round(float(per_tile[0]), 3)}
                    if per_tile.size else None),
        "resolve_start_after_scan_us": round((res - sc[:, 2].max()) / 100.0, 2) if res else None,
        # the time from the previous segment's landing to segment g's landing (g = 0: a new
        # unit's first segment, after the last segment of the previous one)
        "seg_landing_gap_us_by_g": {g: {"median": round(float(np.median(v)), 3), "n": len(v)}
                                    for g, v in sorted(seg_by_g.items())},
        # of that gap: the wave's own work since the previous landing (roll, DMA issue, grab,
        # publish) and its wait for segment g's DMA
        "seg_work_us_by_g": {g: round(float(np.median(v)), 3) for g, v in sorted(work_by_g.items())},
        "seg_wait_us_by_g": {g: round(float(np.median(v)), 3) for g, v in sorted(wait_by_g.items())},
    }
    # per-wave rate (tiles per us of the wave's life) by placement: which waves are slow?
    rate = sc[:, 3] / np.maximum((sc[:, 2] - sc[:, 0]) / 100.0, 1e-3)
    def by(key, n):
        return {int(k): [round(float(rate[key == k].mean()), 4), int((key == k).sum())] for k in range(n)
                if (key == k).any()}
    out["rate_tiles_per_us"] = {"all": [round(float(rate.mean()), 4), round(float(rate.min()), 4),
                                        round(float(rate.max()), 4)],
                                "by_xcc": by(xcc, 8), "by_simd": by(simd, 4), "by_se": by(se, 8),
                                "by_sh": by(sh, 2), "by_cu": by(cu, 16)}
    # waves per (xcc, se, sh, cu, simd) slot: co-residency of the slow ones
    slot = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    _, cnt = np.unique(slot, return_counts=True)
    out["waves_per_simd_hist"] = {int(k): int((cnt == k).sum()) for k in np.unique(cnt)}
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    _, ccnt = np.unique(cu_key, return_counts=True)
    out["waves_per_cu_hist"] = {int(k): int((ccnt == k).sum()) for k in np.unique(ccnt)}
    slow = rate < np.percentile(rate, 10)
    out["slowest10pct_by_xcc"] = {int(k): int((xcc[slow] == k).sum()) for k in range(8)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uniform1k", choices=["uniform1k", "shard8", "zipf10k", "dense1"])
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    os.environ["SYNCR_CDC_TRACE"] = "1"
    lens, idx = table(args.workload, args.shard)
    offs = WL.offsets_of(lens)
    span = int(lens.sum())
    L = syncr_amd.library()
    L.syncr_cdc_dev_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    L.syncr_cdc_dev_trace.restype = ctypes.c_int32
    with syncr_amd.Chunker() as c:
        buf = syncr_amd.DeviceBuffer(c, span)
        try:
            if args.workload == "dense1":
                buf.upload(np.resize(WL.periodic_pattern(), span))
            else:
                buf.gen_corpus(offs, lens, indices=idx)
            c.plan(offs, lens, span)
            info = c.info()
            grid = min(info["scan_grid"], (span + info["tile_bytes"] - 1) // info["tile_bytes"])
            c.launch(buf.ptr)
            c.fetch()
            d = np.zeros(WORDS, np.uint64)
            c.launch(buf.ptr)                                       # the first launch after a host gap
            assert L.syncr_cdc_dev_trace(c.handle, d.ctypes.data, WORDS) == 0
            first = summarize(d, grid)
            for _ in range(args.warmup + args.steps):
                c.launch(buf.ptr)
            assert L.syncr_cdc_dev_trace(c.handle, d.ctypes.data, WORDS) == 0
            last = summarize(d, grid)
        finally:
            buf.free()
    print(json.dumps({"workload": args.workload, "shard": args.shard if args.workload == "shard8" else None,
                      "files": int(lens.size), "bytes": span, "scan_grid": grid, "tile_bytes": info["tile_bytes"],
                      "first_after_gap": first, f"last_of_{args.warmup + args.steps}": last}))


if __name__ == "__main__":
    main()
