#!/bin/bash
# GPU tests; K2t walk four segments per step (x0) against two (x2097152) on C2 and C4s
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="libeazy_amd_x0.so libeazy_amd_x2097152.so" WLS="c2 c4s" REPS=2 bash tools/gpurun/gpurun_lib_ab.sh || exit 1
