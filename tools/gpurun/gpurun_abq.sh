#!/bin/bash
# quick A/B of bench lines without tests: bash tools/gpurun/gpurun_abq.sh WORKLOAD "ENV=V ..." "ENV=V ..." ...
# (each argument after the workload is one arm: space-separated env settings, or "base"); REPS rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/abq
rm -rf $O && mkdir -p $O
W=$1; shift
# arms set environment knobs, which only experiment builds read (make -C eazy_amd exp X=0)
export EZ_LIB=${EZ_LIB:-$GRAFT_REPO_ROOT/eazy_amd/libeazy_amd_x0.so}
for r in $(seq 1 ${REPS:-1}); do
k=0
for ARM in "$@"; do
  k=$((k+1))
  E=""; [ "$ARM" != "base" ] && E="$ARM"
  env $E timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps ${STEPS:-10} --warmup 2 --workload $W ${BARGS:-} > $O/b${r}_$k.json 2> $O/b${r}_$k.err
  rc=$?
  echo "[$r] $ARM rc=$rc $(python3 -c "import json;d=json.load(open('$O/b${r}_$k.json'));print(round(d['value'],2),{k:round(v,3) for k,v in d['kernel_ms'].items()})" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || { tail -5 $O/b${r}_$k.err; exit $rc; }
done
done
