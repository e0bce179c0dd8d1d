"""Mean counter values per kernel from rocprofv3 counter_collection CSVs under a directory.
    python tools/pmc_show.py DIR [kernel-substring]"""
import collections, csv, glob, os, sys
root, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
for d in sorted(glob.glob(os.path.join(root, "*"))):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f: continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if sub in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d), {c: f"{sum(v) / len(v):.4g}" for c, v in sorted(agg.items())})
