import csv, glob, sys, collections
for d in sorted(glob.glob(sys.argv[1] + "/clk_*")):
    f = glob.glob(d + "/*counter_collection.csv")
    if not f: continue
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        if "scan_kernel" not in r["Kernel_Name"]: continue
        k = r["Dispatch_Id"]
        by[k][r["Counter_Name"]] = float(r["Counter_Value"])
        by[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    rows = list(by.values())[1:]
    clk = [x["GRBM_GUI_ACTIVE"] / 8 / x["dur"] / 1e9 for x in rows]
    dur = [x["dur"] * 1e3 for x in rows]
    print(d.split("/")[-1], "dur ms", " ".join(f"{v:.3f}" for v in dur), " clock GHz", " ".join(f"{v:.2f}" for v in clk))
