#!/bin/bash
# GPU tests, then A/B bench lines: bash tools/gpurun/gpurun_ab.sh VAR "v1 v2" "c1 c2"
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ab
rm -rf $O && mkdir -p $O
VAR=$1; VALS=$2; WLS=${3:-c1}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for W in $WLS; do for V in $VALS; do
  env $VAR=$V timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 --workload $W > $O/b_${W}_$V.json 2> $O/b_${W}_$V.err
  rc=$?; echo "$W $VAR=$V rc=$rc $(python3 -c "import json,sys;d=json.load(open('$O/b_${W}_$V.json'));print(round(d['value'],2),d['kernel_ms'])")"; [ $rc -eq 0 ] || exit $rc
done; done
