#!/usr/bin/env python3
"""Per-dispatch durations of the scan (and hash leaf) kernels, in dispatch order,
from a rocprofv3 --kernel-trace CSV (tools/scan_seq.py)."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev_end = None
    for r in rows:
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("cdc::", "")
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (t0 - prev_end) / 1e3 if prev_end else 0.0
        prev_end = t1
        if "scan" in short or "leaf" in short:
            print(f"{short[:40]:40s} {(t1 - t0) / 1e6:8.4f} ms  gap-before {gap:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
