#!/bin/bash
# Round-3 final measurement, part 1: GPU tests, then C1 and C2 (kernel trace for C1, PMC traffic
# passes, bench lines with CPU baselines)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
WLS="c1 c2" bash gpurun_meas.sh
