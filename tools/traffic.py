"""Per-launch HBM traffic of each kernel from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate passes, KB per dispatch).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly
half the bytes of a wide coalesced streaming read (16 B per lane), so it is doubled
for the kernels whose reads are such streams (COALESCED below); the guide does not
validate the factor for scattered reads (the K1 candidate gathers, the lane-per-stream
decoders), so for those the raw figure is the corrected one and the doubled figure is
kept beside it as an upper bound.  WRITE_SIZE is taken as is.  Infinity-Cache hits are
counted (the guide): below ~256 MiB of live data the figures are L2-miss traffic, not HBM.
Output: {kernel_name: {"fetch_raw", "write", "fetch" (corrected), "traffic" (corrected),
"traffic_raw", "traffic_x2" (every fetch doubled), ...}} averaged over dispatches, for
bench.py --traffic-json."""

import collections
import csv
import glob
import json
import os
import sys

root, out = sys.argv[1], sys.argv[2]
# optional: workload streams stream_bytes -> the summary records the kernel-source hash and shape
# it was measured at, so bench.py can use it for later runs of the same kernels (profiles/traffic_<w>.json)
meta = sys.argv[3:6]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        names[k] = 1
    for (k, d, c), v in per.items():
        acc[k][c].append(v * 1024.0)
# kernels whose reads are wide coalesced streams (16 B per lane over consecutive addresses)
COALESCED = ("k3_gather", "k3_scan1", "k3_scan2", "k3_scan3", "kd_copy", "kx_copy")
res = {}
# bench steps profiled: K3's gather runs exactly once per step (pack); kernels a step runs several times
# (K1x's per-round kernels, the general kernel's resume modes) get their per-step sum as well
steps = len(acc["k3_gather"]["FETCH_SIZE"]) if acc.get("k3_gather") and acc["k3_gather"]["FETCH_SIZE"] else None
for k, v in acc.items():
    raw = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"]) if v["FETCH_SIZE"] else None
    write = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) if v["WRITE_SIZE"] else None
    fetch = None if raw is None else (2.0 * raw if k in COALESCED else raw)
    both = raw is not None and write is not None
    tr = fetch + write if both else None
    disp = len(v["FETCH_SIZE"]) or len(v["WRITE_SIZE"])
    per = (lambda t: t * disp / steps if t is not None and steps else None)
    res[k] = {"fetch_raw": raw, "write": write, "fetch": fetch, "fetch_doubled": k in COALESCED,
              "traffic": tr, "traffic_raw": raw + write if both else None, "traffic_x2": 2.0 * raw + write if both else None,
              "dispatches": disp, "per_step": per(tr), "per_step_raw": per(raw + write if both else None),
              "per_step_x2": per(2.0 * raw + write if both else None)}
if meta:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    res = {"source_hash": bench.source_hash(), "workload": meta[0], "streams": int(meta[1]),
           "stream_bytes": int(meta[2]), "kernels": res}
json.dump(res, open(out, "w"), indent=1)
kern = res.get("kernels", res)
print(json.dumps({k: v for k, v in kern.items() if k.startswith("k")}, indent=1))
