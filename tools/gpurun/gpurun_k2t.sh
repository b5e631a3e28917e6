#!/bin/bash
# K2t work loop: decoder GPU tests, C1/C2 A/B of the default K2 against K2t, SQ counters of K2t at C1
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/k2t; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_configs.py -q -x -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpurun/gpurun_abq.sh c1 base EZ_K2=tok || exit 1
BARGS="--no-check" bash tools/gpurun/gpurun_abq.sh c2 base EZ_K2=tok || exit 1
if [ -n "$SQ" ]; then
  EZ_K2=tok SQ_KERNELS="k2_tok k2_ring" bash tools/gpurun/gpurun_sq.sh || exit 1
fi
