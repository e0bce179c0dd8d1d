#!/usr/bin/env python3
"""Summarise a tools/prof.sh run (gpurun_out/prof_<tag>/) into profiles/.

Writes
  profiles/<tag>_kernel_stats.csv     rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_bench_trace.json     the bench JSON line of the traced run
  profiles/<tag>_dispatches.json      scan / BLAKE3-leaf durations per dispatch, in order, and the
                                      mean over the bench's timed window vs over every launch
  profiles/<tag>_pmc_traffic.json     HBM bytes per launch: scan (main) and every other kernel
  profiles/<tag>_pmc_sq.json          per scan dispatch: shader clock and SQ instruction counters

Read bytes come from the L2->EA request-size counters (pass 2, prof.sh r02+):
64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B + 32*TCC_EA0_RDREQ_32B.  gfx950's
FETCH_SIZE formula weights 128-byte requests by TCC_BUBBLE, which reads 0 on
gfx950, so FETCH_SIZE counts every 128-byte request as 64 B (exactly half on
streaming reads); profiles/r02_fetch_calibration.json measures both on known
byte counts (tools/ubench_fetch.hip).  Older runs (FETCH_SIZE pass) are doubled,
which is exact only when every request is 128 B.  Write bytes: WRITE_SIZE, own pass.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0].replace("void ", "")
    if "cdc_scan_st_kernel" in n:
        return "cdc::cdc_scan_st_kernel"
    if "cdc_scan_kernel" in n:
        return "cdc::cdc_scan_kernel"
    if "b3_leaf_kernel" in n:
        return "cdc::b3_leaf_kernel"
    return n


def counters(path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def bench_line(log):
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def dispatches(trace_csv, line, k="cdc::cdc_scan_kernel"):
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    scans = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if short(r["Kernel_Name"]) == k]
    leaf = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
            if short(r["Kernel_Name"]) == "cdc::b3_leaf_kernel"]
    w, k = (line or {}).get("warmup", 0), (line or {}).get("steps", 0)
    timed = scans[w:w + k]                     # bench.py: W warm-up scans, then the K timed ones
    mean = lambda v: sum(v) / len(v) if v else None   # noqa: E731
    return {
        "scan_ms_per_dispatch": [round(x, 4) for x in scans],
        "scan_ms_mean_all": mean(scans), "scan_launches": len(scans),
        "scan_ms_mean_timed_window": mean(timed), "timed_window": [w, w + k],
        "bench_line_scan_ms": (line or {}).get("roofline", {}).get("kernel_ms"),
        "leaf_ms_per_dispatch": [round(x, 4) for x in leaf], "leaf_ms_mean": mean(leaf),
        "bench_line_scan_ms_hip_events": (line or {}).get("roofline", {}).get("kernel_ms_hip_events"),
        "note": "rocprofv3 kernel-trace durations; the bench line's kernel_ms is the device-clock mean over the "
                "same timed window (syncr_cdc_set_timing mode 4), kernel_ms_hip_events its event-pair cross-check "
                "on the K steps after it (profiling adds a few % per dispatch)",
    }


def main(tag, src=None):
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    b = bench_line(os.path.join(src, "bench_trace.log"))
    json.dump(b, open(os.path.join(dst, f"{tag}_bench_trace.json"), "w"), indent=1)
    f = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    # the headline's scan kernel: stream tiles on large batches (round 4), else the tile scan
    k = "cdc::cdc_scan_st_kernel" if any(kk[0] == "cdc::cdc_scan_st_kernel" for kk in f) else "cdc::cdc_scan_kernel"
    json.dump(dispatches(os.path.join(src, "trace", "run_kernel_trace.csv"), b, k),
              open(os.path.join(dst, f"{tag}_dispatches.json"), "w"), indent=1)
    w = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    fb = bench_line(os.path.join(src, "bench_fetch.log")) or {}
    span = fb.get("config", {}).get("bytes_per_gpu")
    mean = lambda v: sum(v) / len(v) if v else 0.0   # noqa: E731
    sized = any(c == "TCC_EA0_RDREQ_128B" for _, c in f)

    def read_bytes(kname):
        if sized:
            v = {c: mean(f.get((kname, c), [])) for c in ("TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B",
                                                          "TCC_EA0_RDREQ_128B")}
            if not f.get((kname, "TCC_EA0_RDREQ_128B")):
                return None
            return 32 * v["TCC_EA0_RDREQ_32B"] + 64 * v["TCC_EA0_RDREQ_64B"] + 128 * v["TCC_EA0_RDREQ_128B"]
        fv = f.get((kname, "FETCH_SIZE"), [])
        return 2 * 1024 * mean(fv) if fv else None

    def hbm(kname):
        r = read_bytes(kname)
        return None if r is None else r + 1024 * mean(w.get((kname, "WRITE_SIZE"), []))

    read_b = read_bytes(k)
    write_kib = mean(w[(k, "WRITE_SIZE")])
    scan_hbm = hbm(k)
    kernels = sorted({kk[0] for kk in f})
    out = {
        "kernel": k, "workload": fb.get("config", {}).get("workload", "").split(":")[0],
        # the stream-tile geometry the library reported for the headline launches
        "st_segments": (fb.get("roofline", {}).get("scan_schedule") or {}).get("st_segments"),
        "run_bytes": fb.get("config", {}).get("engine", {}).get("run_bytes"),
        "span": span, "read_bytes": int(read_b), "write_size_kib": write_kib,
        "hbm_bytes_per_launch": int(scan_hbm), "algorithmic_bytes_per_launch": span,
        "traffic_over_algorithmic": (scan_hbm / span) if span else None,
        "correction": ("bytes = 32*TCC_EA0_RDREQ_32B + 64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B + WRITE_SIZE*1024 "
                       "(gfx950 FETCH_SIZE counts 128-byte requests as 64 B: profiles/r02_fetch_calibration.json)"
                       if sized else "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (exact when every request is 128 B)"),
        "scope": "L2 -> EA (fabric) requests: Infinity Cache hits are included, so this bounds HBM bytes from above",
        "source": (f"rocprofv3 --pmc TCC_EA0_RDREQ_{{32B,64B,128B}} TCC_EA0_RDREQ / --pmc WRITE_SIZE (separate passes), "
                   f"tools/prof.sh {tag}" if sized else
                   f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/prof.sh {tag}"),
        "per_kernel_hbm_bytes": {kn: int(hbm(kn)) for kn in kernels if hbm(kn) is not None},
        "per_kernel_traffic_over_span": {kn: round(hbm(kn) / span, 4) for kn in kernels
                                         if hbm(kn) is not None and span},
    }
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    sq_csv = os.path.join(src, "pmc_sq", "run_counter_collection.csv")
    if os.path.exists(sq_csv):
        per = defaultdict(dict)
        allk = defaultdict(lambda: defaultdict(dict))      # kernel -> dispatch -> counters
        for r in csv.DictReader(open(sq_csv)):
            kn = short(r["Kernel_Name"])
            a = allk[kn][int(r["Dispatch_Id"])]
            a[r["Counter_Name"]] = a.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            a["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if kn != k:
                continue
            d = per[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        rows = []
        for disp in sorted(per):
            d = per[disp]
            clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / (d["dur_ms"] / 1e3) / 1e9 if d.get("dur_ms") else None
            rows.append({"dispatch": disp, "ms": round(d["dur_ms"], 4), "clock_ghz": round(clk, 3) if clk else None,
                         **{c: d[c] for c in d if c.startswith("SQ_")}})
        per_kernel = {}
        for kn, disp in allk.items():
            ds = list(disp.values())
            m = {c: sum(d.get(c, 0.0) for d in ds) / len(ds) for c in ds[0] if c.startswith(("SQ_", "GRBM_"))}
            ms = sum(d["dur_ms"] for d in ds) / len(ds)
            act = m.get("SQ_ACTIVE_INST_VALU", 0.0)
            wc = m.get("SQ_WAVE_CYCLES", 0.0)
            per_kernel[kn] = {"dispatches": len(ds), "ms_mean": round(ms, 4), **{c: round(v, 1) for c, v in m.items()},
                              "valu_active_over_wave_cycles": round(act / wc, 4) if wc else None,
                              "wait_any_over_wave_cycles": round(m.get("SQ_WAIT_ANY", 0.0) / wc, 4) if wc else None}
        json.dump({"kernel": k, "source": f"tools/prof.sh {tag} pass 4", "per_dispatch": rows,
                   "per_kernel_mean": per_kernel,
                   "units": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles (MI355X_MICROARCH.md); "
                            "clock = GRBM_GUI_ACTIVE / 8 XCDs / duration"},
                  open(os.path.join(dst, f"{tag}_pmc_sq.json"), "w"), indent=1)
    print(json.dumps({kk: v for kk, v in out.items() if kk != "per_kernel_hbm_bytes"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02", sys.argv[2] if len(sys.argv) > 2 else None)
