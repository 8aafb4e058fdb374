#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs of tools/profile.sh per kernel (sum over dispatches, per dispatch)."""
import csv, collections, glob, sys

root = sys.argv[1]
for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    meta = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("hlc::(anonymous namespace)::", "").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        meta[k] = f"vgpr={r['VGPR_Count']} sgpr={r['SGPR_Count']} scratch={r['Scratch_Size']} lds={r['LDS_Block_Size']} grid={r['Grid_Size']}"
    print("==", f.split("/")[-2])
    for k in sorted(agg, key=lambda k: -sum(agg[k].values())):
        if not any(x in k for x in ("recover", "prehash", "chain", "tables")):
            continue
        nd = len(disp[k])
        vals = " ".join(f"{c}={v / nd:.4g}" for c, v in sorted(agg[k].items()))
        print(f"  {k} [{nd} dispatches, {meta[k]}] per dispatch: {vals}")
