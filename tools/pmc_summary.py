#!/usr/bin/env python3
"""Summarise a tools/prof.sh run (gpurun_out/prof_<tag>/) into profiles/.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc_traffic.json   HBM bytes per cdc_scan_kernel launch
  profiles/<tag>_bench_trace.json   the bench JSON line of the traced run

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB
and collected in separate passes; on gfx950 FETCH_SIZE reports exactly half of
the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "cdc_scan_kernel" in name:
            name = "cdc::cdc_scan_kernel"
        if "b3_leaf_kernel" in name:
            name = "cdc::b3_leaf_kernel"
        agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def bench_line(log):
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def main(tag, src=None):
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    b = bench_line(os.path.join(src, "bench_trace.log"))
    json.dump(b, open(os.path.join(dst, f"{tag}_bench_trace.json"), "w"), indent=1)
    f = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    w = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    k = "cdc::cdc_scan_kernel"
    fetch_kib = sum(f[(k, "FETCH_SIZE")]) / len(f[(k, "FETCH_SIZE")])
    write_kib = sum(w[(k, "WRITE_SIZE")]) / len(w[(k, "WRITE_SIZE")])
    fb = json.load(open(os.path.join(dst, f"{tag}_bench_trace.json"))) if b else {}
    span = fb.get("config", {}).get("bytes_per_gpu")
    hbm = 2 * fetch_kib * 1024 + write_kib * 1024
    out = {
        "kernel": k, "workload": fb.get("config", {}).get("workload", "").split(":")[0],
        "run_bytes": fb.get("config", {}).get("engine", {}).get("run_bytes"),
        "span": span, "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
        "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": span,
        "traffic_over_algorithmic": (hbm / span) if span else None,
        "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halves wide streaming reads)",
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/prof.sh {tag}",
        "other_kernels": {kk[0]: sum(v) / len(v) for kk, v in {**f, **w}.items() if kk[0] != k},
        "per_kernel_hbm_bytes": {
            kk[0]: int(2 * 1024 * sum(v) / len(v) + 1024 * (sum(w[(kk[0], "WRITE_SIZE")]) / max(len(w[(kk[0], "WRITE_SIZE")]), 1)))
            for kk, v in f.items() if kk[1] == "FETCH_SIZE"},
    }
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else None)
