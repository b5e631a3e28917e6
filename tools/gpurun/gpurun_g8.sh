#!/bin/bash
# 8-lane k1_lean groups: parity on the batch tests (experiment build, EZ_K1S_G=8), then tools/exp.txt
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EZ_LIB=eazy_amd/libeazy_amd_x0.so EZ_K1S_G=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_configs.py -q -m gpu -k "auto or c1 or C1 or log or edge or ragged or tiny" --timeout 300 --timeout-method thread > gpurun_out/g8_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/g8_tests.log | tail -8; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/exp
bash tools/gpurun/exp.sh tools/exp.txt
