#!/bin/bash
# C1 kernel-trace stats, alternating: x0 (candidate from two loads, cap 24 - r) and x65536 (three
# loads, cap 24), three rounds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab7; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do
for arm in x0 x65536; do
  EZ_LIB=$R/eazy_amd/libeazy_amd_$arm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$arm$rep -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 --workload c1 > $O/$arm$rep.log 2>&1 || { tail -5 $O/$arm$rep.log; exit 1; }
  python3 - <<PY
import csv,glob
f=glob.glob("$O/$arm$rep/**/*kernel_stats.csv",recursive=True)[0]
print("$arm", *[r["Name"].split("(")[0].split("::")[-1][:12]+" "+str(round(float(r["AverageNs"])/1e3,1)) for r in csv.DictReader(open(f)) if "k1_lean" in r["Name"] or "k1_emit" in r["Name"]])
PY
done
done
