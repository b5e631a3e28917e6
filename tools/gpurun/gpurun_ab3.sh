#!/bin/bash
# A/B: K2t adaptive resolution (x0 vs x8192) on C2/C4s; kernel-trace stats of C1 for x0, x32768 (k1_lean
# record stores to two slots, timing only) and x0 at 4 waves per SIMD (LDS padding)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIBS="libeazy_amd_x0.so libeazy_amd_x8192.so" WLS="c2 c4s" REPS=2 bash tools/gpurun/gpurun_lib_ab.sh || exit 1
O=$R/gpurun_out/ab3; rm -rf $O; mkdir -p $O
for arm in x0 x32768 pad; do
  L=$arm; E=""; [ $arm = pad ] && { L=x0; E="EZ_K1S_LDSPAD=2048"; }
  env EZ_LIB=$R/eazy_amd/libeazy_amd_$L.so $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$arm -o run -- python3 bench.py --no-cpu --no-e2e --no-check --steps 10 --warmup 2 --workload c1 > $O/$arm.log 2>&1 || { tail -5 $O/$arm.log; exit 1; }
  python3 - <<PY
import csv,glob
f=glob.glob("$O/$arm/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r["Name"].split("(")[0].replace("ez::(anonymous namespace)::","")
    if "k1_" in n or "k2_" in n: print("$arm", n, round(float(r["AverageNs"])/1e3,1), "us")
PY
done
