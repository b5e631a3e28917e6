#!/bin/bash
# round 5: decoder A/B over the workloads (tools/exp.txt), after the K2j GPU tests
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_stream.py -q -m gpu --timeout 300 --timeout-method thread -k "k2j or whole or k2t or decoder" > gpurun_out/t2.log 2>&1
rc=$?; tail -5 gpurun_out/t2.log | grep -v "^$"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpurun/exp.sh tools/exp.txt
