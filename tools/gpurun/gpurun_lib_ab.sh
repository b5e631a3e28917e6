#!/bin/bash
# A/B of whole libraries on bench lines: LIBS="libeazy_amd_x0.so libeazy_amd.so" WLS="c2 c4s" bash tools/gpurun/gpurun_lib_ab.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/libab
rm -rf $O && mkdir -p $O
for r in $(seq 1 ${REPS:-1}); do
for L in $LIBS; do
  for W in $WLS; do
    EZ_LIB=$GRAFT_REPO_ROOT/eazy_amd/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps ${STEPS:-3} --warmup 1 --workload $W ${BARGS:-} > $O/${r}_${L}_${W}.json 2> $O/${r}_${L}_${W}.err
    rc=$?
    echo "[$r] $L $W rc=$rc $(python3 -c "import json;d=json.load(open('$O/${r}_${L}_${W}.json'));print(round(d['value'],2),{k:round(v,3) for k,v in d['kernel_ms'].items()})" 2>&1 | tail -1)"
    [ $rc -eq 0 ] || { tail -5 $O/${r}_${L}_${W}.err; exit $rc; }
  done
done
done
