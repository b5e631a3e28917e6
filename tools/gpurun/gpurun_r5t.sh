#!/bin/bash
# round 5: the whole GPU suite (no -x: every failure listed), then tools/exp.txt
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -15; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
rm -rf gpurun_out/exp
bash tools/gpurun/exp.sh tools/exp.txt
