#!/usr/bin/env python3
"""Per-step breakdown of a tools/legs_trace.py run under rocprofv3
--kernel-trace: the timed window (steps W .. W+K-1 of time_steps) split into
the scan, each post-scan kernel and the gaps between them (us, means over the
window), plus the step period (scan start to next scan start).

    python tools/legs_trace_show.py <kernel_trace.csv> <steps K> <warmup W> [bytes]
"""
import csv
import json
import sys
from collections import defaultdict


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("cdc::", "")
    return n.split("<")[0]


def main():
    path, K, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    nbytes = int(sys.argv[4]) if len(sys.argv) > 4 else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    rows = [r for r in rows if r[0].startswith(("cdc_", "b3_"))]
    SCANS = ("cdc_scan_kernel", "cdc_scan_st_kernel")           # the scan a step starts with (any schedule)
    rows = [("scan" if r[0] in SCANS else r[0], r[1], r[2]) for r in rows]
    starts = [k for k, r in enumerate(rows) if r[0] == "scan"]
    steps = []
    for j, k in enumerate(starts):
        end = starts[j + 1] if j + 1 < len(starts) else len(rows)
        steps.append(rows[k:end])
    window = steps[W:W + K]
    dur = defaultdict(list)
    gap = defaultdict(list)
    period = []
    for j, st in enumerate(window):
        t0 = st[0][1]
        for a, b in zip(st, st[1:]):
            gap[f"{a[0]} -> {b[0]}"].append((b[1] - a[2]) / 1e3)
        for name, s, e in st:
            dur[name].append((e - s) / 1e3)
        # the next step inside the window only: the window's last launch is followed by the
        # host's synchronize (and the phase-timed launches), not by a timed step
        nxt = steps[W + j + 1][0][1] if j + 1 < len(window) else None
        if nxt:
            period.append((nxt - t0) / 1e3)
            gap["last -> next scan"].append((nxt - st[-1][2]) / 1e3)
        dur["step (scan start .. last kernel end)"].append((st[-1][2] - t0) / 1e3)
    mean = lambda v: round(sum(v) / len(v), 2) if v else None   # noqa: E731
    out = {"steps_in_window": len(window), "kernel_us": {k: mean(v) for k, v in dur.items()},
           "gap_us": {k: mean(v) for k, v in gap.items()}, "period_us": mean(period),
           "scan_us_each": [round(v, 1) for v in dur["scan"]]}
    if nbytes:
        out["scan_frac_8tbs"] = round(nbytes / (out["kernel_us"]["scan"] / 1e6) / 8e12, 4)
        if out["period_us"]:
            out["period_frac_8tbs"] = round(nbytes / (out["period_us"] / 1e6) / 8e12, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
