#!/bin/bash
# round 5: GPU tests (all of them, a failure does not stop the measurements unless it crashed or
# timed out), then the lone-stream K2t / K2j timings and the K1 A/B matrix of tools/exp.txt
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; tail -25 gpurun_out/t1.log | grep -v "^$"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
for k in t j; do
  timeout -k 10 120 python tools/lone_k2t.py 16 --check --kind $k || exit 1
done
bash tools/gpurun/exp.sh tools/exp.txt
