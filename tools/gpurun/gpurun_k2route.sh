#!/bin/bash
# K2 routing A/B for long-slot batches: the automatic choice against K2r forced (EZ_K2=ring), 1 GiB
# of log-like streams per size: bash tools/gpurun/gpurun_k2route.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/k2route; rm -rf $O; mkdir -p $O
TOTAL=$((1 << 30))
for Z in ${SZ:-65536 131072 262144}; do
  N=$((TOTAL / Z))
  for V in auto ring; do
    E=""; [ $V = ring ] && E="EZ_K2=ring"
    env $E timeout -k 10 300 python3 bench.py --workload c2 --stream-bytes $Z --streams $N --no-e2e --no-cpu --steps 5 --warmup 1 > $O/b_${Z}_$V.json 2> $O/b_${Z}_$V.err
    rc=$?; echo "size $Z $V rc=$rc $(python3 -c "import json;d=json.load(open('$O/b_${Z}_$V.json'));print(round(d['decompress_GiBps'],1),d['kernel_ms'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
