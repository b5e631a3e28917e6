#!/bin/bash
# A/B of library builds (EZ_LIB) with extra env and bench args, no round-trip checks (ablation builds):
# LIBS="a.so b.so" WL=c1 ENVS="EZ_K2=tok" bash tools/gpurun/gpurun_libab2.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/libab2; mkdir -p $O
for L in $LIBS; do
  env $ENVS EZ_LIB=$GRAFT_REPO_ROOT/eazy_amd/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-check --steps ${STEPS:-10} --warmup 2 --workload ${WL:-c1} > $O/${WL:-c1}_$L.json 2> $O/${WL:-c1}_$L.err
  rc=$?; echo "$WL $L rc=$rc $(python3 -c "import json;d=json.load(open('$O/${WL:-c1}_$L.json'));print(round(d['value'],2),d['kernel_ms'])" 2>&1 | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
