#!/bin/bash
# K1c / K2 routing: the K1c, K1x and config tests, then tools/exp.txt
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_k1c.py tests/test_gpu_configs.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/k1c3_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/k1c3_tests.log | tail -8; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/exp
bash tools/gpurun/exp.sh tools/exp.txt
