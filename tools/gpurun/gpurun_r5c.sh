#!/bin/bash
# round 5: K1 A/B matrix (tools/exp.txt), then the SQ counters of the default build at C1
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_configs.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?; tail -3 gpurun_out/t3.log | grep -v "^$"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpurun/exp.sh tools/exp.txt || exit 1
bash tools/gpurun/gpurun_sq.sh
