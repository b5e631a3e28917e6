"""Aggregate rocprofv3 --pmc CSV passes per kernel (mean per dispatch)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "ez::"
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        k = k.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        nd = len(disp[k])
        print(f.split("/")[-2], k, "dispatches", nd, {c: f"{x / nd:.4g}" for c, x in v.items()})
