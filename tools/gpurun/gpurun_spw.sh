#!/bin/bash
# K1L streams-per-wave A/B on the long-stream configs: GPU tests, then C2 / C4s bench lines
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/spw; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for W in ${WLS:-c2 c4s}; do for V in ${VALS:-4 0}; do
  env EZ_K1L_SPW=$V timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workload $W > $O/b_${W}_$V.json 2> $O/b_${W}_$V.err
  rc=$?; echo "$W spw=$V rc=$rc $(python3 -c "import json;d=json.load(open('$O/b_${W}_$V.json'));print(round(d['value'],3),round(d['compress_GiBps'],3),d['kernel_ms'])")"; [ $rc -eq 0 ] || exit $rc
done; done
