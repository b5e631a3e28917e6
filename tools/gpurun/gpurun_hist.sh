#!/bin/bash
# k1_lean's acceptor-lane histogram at C1 (experiment build X=65536)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EZ_LIB=eazy_amd/libeazy_amd_x65536.so timeout -k 10 200 python bench.py --workload c1 --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/hist.json 2> gpurun_out/hist.err
rc=$?; grep "lean windows" gpurun_out/hist.err | head -3; exit $rc
