#!/bin/bash
# GPU tests at the current tree, then the C1 measurement (kernel trace, PMC traffic, bench line),
# then an A/B of experiment libraries (LIBS, WLS) when LIBS is set
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$MEAS" ]; then WLS="$MEAS" bash gpurun_meas.sh || exit 1; fi
if [ -n "$LIBS" ]; then bash tools/gpurun/gpurun_lib_ab.sh || exit 1; fi
