#!/bin/bash
# GPU tests; C1 kernel-trace stats: x0 (k1_lean on two candidate loads, LDS token writer) against
# x0 with k1_emit (EZ_K1E_LDS=0); then the bench line
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
O=$R/gpurun_out/ab6; rm -rf $O; mkdir -p $O
for rep in 1 2; do
for arm in lds old; do
  E=""; [ $arm = old ] && E="EZ_K1E_LDS=0"
  env EZ_LIB=$R/eazy_amd/libeazy_amd_x0.so $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$arm$rep -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 --workload c1 > $O/$arm$rep.log 2>&1 || { tail -5 $O/$arm$rep.log; exit 1; }
  python3 - <<PY
import csv,glob
f=glob.glob("$O/$arm$rep/**/*kernel_stats.csv",recursive=True)[0]
print("$arm", *[r["Name"].split("(")[0].replace("ez::(anonymous namespace)::","").replace("void ","")[:16]+" "+str(round(float(r["AverageNs"])/1e3,1)) for r in csv.DictReader(open(f)) if "k1_" in r["Name"] or "k2_ring" in r["Name"] or "k3_" in r["Name"]])
PY
done
done
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --workload c1 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],2), d['kernel_ms'])"
