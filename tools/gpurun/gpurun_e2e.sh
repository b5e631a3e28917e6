#!/bin/bash
# overlapped host-memory (PCIe-inclusive) measurement at several chunk counts
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/e2e
rm -rf $O && mkdir -p $O
for C in ${1:-2 4 8}; do
  timeout -k 10 300 python3 bench.py --no-cpu --steps 5 --warmup 1 --e2e-chunks $C > $O/b_$C.json 2> $O/b_$C.err
  rc=$?; echo "chunks $C rc=$rc $(python3 -c "import json;d=json.load(open('$O/b_$C.json'));print(d['e2e'])")"; [ $rc -eq 0 ] || { tail -5 $O/b_$C.err; exit $rc; }
done
