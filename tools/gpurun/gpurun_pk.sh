#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pk
for wl in c2 c4s; do
EZ_LIB=eazy_amd/libeazy_amd_x0.so EZ_K1C_PASSES=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk/$wl -o run -- python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu --no-e2e --no-check > gpurun_out/pk/$wl.log 2>&1 || exit 1
f=$(find gpurun_out/pk/$wl -name "*kernel_stats.csv" | head -1); head -30 "$f" | cut -d, -f1-4
done
