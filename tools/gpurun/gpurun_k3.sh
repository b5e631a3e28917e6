#!/bin/bash
# GPU tests, then the C4/C2 bench lines (K3 gather split experiment)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/k3
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for W in c4 c2 c1; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1 --workload $W > $O/bench_$W.json 2> $O/bench_$W.err
  rc=$?; echo "bench $W rc=$rc"; cat $O/bench_$W.json; [ $rc -eq 0 ] || exit $rc
done
