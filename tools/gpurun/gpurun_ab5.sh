#!/bin/bash
# GPU tests; C1 kernel-trace stats: x0 against timing builds with fewer candidate loads (x65536: no
# third dword; x131072: one 16-byte load) and against K2r reloading every header (x262144)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
O=$R/gpurun_out/ab5; rm -rf $O; mkdir -p $O
for rep in 1 2; do
for arm in x0 x65536 x131072 x262144; do
  EZ_LIB=$R/eazy_amd/libeazy_amd_$arm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$arm$rep -o run -- python3 bench.py --no-cpu --no-e2e --no-check --steps 10 --warmup 2 --workload c1 > $O/$arm$rep.log 2>&1 || { tail -5 $O/$arm$rep.log; exit 1; }
  python3 - <<PY
import csv,glob
f=glob.glob("$O/$arm$rep/**/*kernel_stats.csv",recursive=True)[0]
print("$arm", *[r["Name"].split("(")[0].replace("ez::(anonymous namespace)::","")[-10:]+" "+str(round(float(r["AverageNs"])/1e3,1)) for r in csv.DictReader(open(f)) if "k1_lean" in r["Name"] or "k2_ring" in r["Name"]])
PY
done
done
