#!/bin/bash
# kernel-time breakdown (rocprofv3 --kernel-trace --stats) of the given workloads (WLS="name:args|...")
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pk
IFS='|' read -ra specs <<< "${WLS:-c4s:--workload c4s}"
for spec in "${specs[@]}"; do
wl=${spec%%:*}; args=${spec#*:}
rm -rf gpurun_out/pk/$wl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk/$wl -o run -- python bench.py $args --steps 2 --warmup 1 --no-cpu --no-e2e --no-check > gpurun_out/pk/$wl.log 2>&1 || exit 1
done
