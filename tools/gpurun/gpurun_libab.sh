#!/bin/bash
# A/B of library builds (EZ_LIB) on one workload: LIBS="a.so b.so" WL=c1 STEPS=10 bash tools/gpurun/gpurun_libab.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/libab; rm -rf $O; mkdir -p $O
for L in ${LIBS:-libeazy_amd_s_max-ilp.so libeazy_amd.so libeazy_amd_s_max-memory-clause.so libeazy_amd_s_max-ilp.so libeazy_amd.so}; do
  EZ_LIB=$GRAFT_REPO_ROOT/eazy_amd/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps ${STEPS:-10} --warmup 2 --workload ${WL:-c1} > $O/${WL:-c1}_$L.json 2> $O/${WL:-c1}_$L.err
  rc=$?; echo "$L rc=$rc $(python3 -c "import json;d=json.load(open('$O/${WL:-c1}_$L.json'));print(round(d['value'],2),d['kernel_ms'])")"; [ $rc -eq 0 ] || exit $rc
done
