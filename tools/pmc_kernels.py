#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc run's counters (one row per kernel:
dispatches and the mean of every counter over them).

    python tools/pmc_kernels.py <dir>/run_counter_collection.csv [kernel-substring]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    agg = defaultdict(lambda: defaultdict(list))
    disp = defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if len(sys.argv) > 2 and sys.argv[2] not in k:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp[k]))
    out = {k: {"dispatches": len(disp[k]), **{c: round(sum(v) / len(v), 1) for c, v in cs.items()}}
           for k, cs in agg.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
