"""Sum rocprofv3 counter_collection.csv files per kernel (averaged over dispatches):
python tools/pmc_sum.py gpurun_out/pmc/p*/run_counter_collection.csv [kernel-substring]"""
import csv
import sys
from collections import defaultdict

files = [f for f in sys.argv[1:] if f.endswith(".csv")]
filt = [a for a in sys.argv[1:] if not a.endswith(".csv")]
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        if filt and not any(x in k for x in filt):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        n = len(disp[k][c])
        print(f"   {c:24s} {v / n:16.0f}   (per dispatch, {n} dispatches)")
