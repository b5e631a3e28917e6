"""Per-step kernel times from tools/gpurun/gpurun_pk.sh's rocprofv3 stats: python tools/pk_summary.py NAME..."""
import csv
import re
import sys

for wl in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"gpurun_out/pk/{wl}/run_kernel_stats.csv")))
    print(wl)
    for r in rows[:18]:
        m = re.search(r"::(\w+(<[^>]*>)?)\(", r["Name"])
        print(f"  {(m.group(1) if m else r['Name'][:30]):34s} calls {r['Calls']:>5} {int(r['TotalDurationNs']) / 1e6 / 3:8.3f} ms/step")
