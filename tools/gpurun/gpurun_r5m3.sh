#!/bin/bash
# round 5 measurement, part 3: C4s's bench line again (K1 / K2 stage sums now count K1c, the wide
# token writer and K2j), the handle path / Reader rates with a workspace-sizing warm-up
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/meas
timeout -k 10 600 python3 bench.py --traffic-json profiles/traffic_c4s.json --workload c4s --steps 10 --no-e2e > gpurun_out/meas/c4s.json 2> gpurun_out/meas/c4s.err || exit 1
echo "c4s ok"
timeout -k 10 400 python tests/perf_handle.py > gpurun_out/perf_handle.json 2> gpurun_out/perf_handle.err || exit 1
echo "perf_handle ok"
