#!/bin/bash
# round 5: GPU tests, then the K1 persistent-group A/B and the lone-stream K2t / K2j timings
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; tail -15 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
for k in t j; do
  timeout -k 10 120 python tools/lone_k2t.py 16 --check --kind $k || exit 1
done
bash tools/gpurun/exp.sh tools/exp.txt
