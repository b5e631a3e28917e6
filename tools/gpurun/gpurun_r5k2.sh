#!/bin/bash
# round 5: K1c parity tests, then the A/B lines of tools/exp.txt with K1c's per-pass verdicts
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_k1c.py -x -v --timeout 200 --timeout-method thread > gpurun_out/k1c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/k1c_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/exp
bash tools/gpurun/exp.sh tools/exp.txt || exit 1
for f in gpurun_out/exp/e*.err; do echo "$f: $(grep "K1c pass" $f | tail -8 | sort -u | tr '\n' '|')"; done
