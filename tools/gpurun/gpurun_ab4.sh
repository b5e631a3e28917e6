#!/bin/bash
# GPU tests; C1 kernel-trace stats: x0 (12-bit tables), x0 with u16 tables (EZ_K1S_T12=0), x32768
# (record stores to two slots, timing only); K2t adaptive resolution A/B (x0 vs x8192) on C2/C4s
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
O=$R/gpurun_out/ab4; rm -rf $O; mkdir -p $O
for rep in 1 2; do
for arm in t12 t16 norec; do
  L=x0; E=""; [ $arm = t16 ] && E="EZ_K1S_T12=0"; [ $arm = norec ] && L=x32768
  env EZ_LIB=$R/eazy_amd/libeazy_amd_$L.so $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$arm$rep -o run -- python3 bench.py --no-cpu --no-e2e --no-check --steps 10 --warmup 2 --workload c1 > $O/$arm$rep.log 2>&1 || { tail -5 $O/$arm$rep.log; exit 1; }
  python3 - <<PY
import csv,glob
f=glob.glob("$O/$arm$rep/**/*kernel_stats.csv",recursive=True)[0]
print("$arm", *[r["Name"].split("(")[0].replace("ez::(anonymous namespace)::","")[:14]+" "+str(round(float(r["AverageNs"])/1e3,1)) for r in csv.DictReader(open(f)) if "k1_" in r["Name"] or "k2_" in r["Name"]])
PY
done
done
LIBS="libeazy_amd_x0.so libeazy_amd_x8192.so" WLS="c2 c4s" REPS=2 bash tools/gpurun/gpurun_lib_ab.sh || exit 1
