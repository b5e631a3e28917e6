#!/bin/bash
# GPU tests, then K1 A/B (one-atomic visit vs DPP search) on C1 and K2t A/B (round-start copy
# resolution vs batches only) on C2 and C4s, experiment libraries
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpurun/gpurun_abq.sh c1 base EZ_K1S_MSK=0 || exit 1
LIBS="libeazy_amd_x8192.so libeazy_amd_x0.so" WLS="c2 c4s" REPS=2 bash tools/gpurun/gpurun_lib_ab.sh || exit 1
