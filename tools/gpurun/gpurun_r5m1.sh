#!/bin/bash
# round 5 measurement, part 1: the GPU test suite, then per-workload traffic + bench lines (c1 c2 c4 c4h)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log | grep -v "^$"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
WLS="${WLS:-c1 c2 c4 c4h}" bash tools/gpurun/gpurun_meas.sh
