#!/bin/bash
# GPU tests, then a 2-rank C3 bench on the box's one card through bench.py's own launcher
# (both ranks on cuda:0; RCCL size all-gather and P2P payload gather end to end)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/t2
rm -rf $O && mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -q -x -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/gpu_tests.log | grep -v "^$" | tail -8; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python3 bench.py --gpus 2 --workload c3 --streams ${C3_STREAMS:-131072} --steps 5 --warmup 1 --cpu-seconds 4 > $O/c3_2rank.json 2> $O/c3_2rank.err
rc=$?; echo "c3 2-rank rc=$rc"; tail -c 1500 $O/c3_2rank.json; tail -5 $O/c3_2rank.err
exit $rc
