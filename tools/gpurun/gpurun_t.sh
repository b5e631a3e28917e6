#!/bin/bash
# GPU tests (selection via TESTS, default all -m gpu), then quick A/B arms of the bench (gpurun_abq.sh args)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/t
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -q -x -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/gpu_tests.log | grep -v "^$" | tail -8; [ $rc -eq 0 ] || exit $rc
[ $# -gt 0 ] || exit 0
bash tools/gpurun/gpurun_abq.sh "$@"
exit $?
