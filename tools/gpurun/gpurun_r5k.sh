#!/bin/bash
# round 5: K1c parity tests, then K1c against K1L (A/B lines in tools/exp.txt)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_k1c.py -x -v --timeout 200 --timeout-method thread > gpurun_out/k1c_tests.log 2>&1
rc=$?; tail -12 gpurun_out/k1c_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpurun/exp.sh tools/exp.txt; grep -h "K1c pass" gpurun_out/exp/*.err | sort | uniq -c | head -40
