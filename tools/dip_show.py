#!/usr/bin/env python3
"""Per-dispatch durations (ms) in launch order from a rocprofv3 kernel trace,
grouped into runs of one kernel name:  python tools/dip_show.py TRACE_DIR [substr ...]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
subs = sys.argv[2:] or ["cdc_scan", "reduce"]
f = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
runs = []
for r in rows:
    name = r["Kernel_Name"]
    key = next((s for s in subs if s in name), None)
    if key is None:
        continue
    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if runs and runs[-1][0] == key:
        runs[-1][1].append(ms)
    else:
        runs.append((key, [ms]))
for key, v in runs:
    print(f"{key:10s} n={len(v):3d}  " + " ".join(f"{m:.3f}" for m in v))
