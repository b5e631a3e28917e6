#!/bin/bash
# round 5 measurement, part 2: C3 on one GPU (traffic + bench line), the handle-path / Reader rates,
# the lone-stream decoders, the HBM sweep over stream sizes
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
WLS="c3" bash tools/gpurun/gpurun_meas.sh || exit $?
timeout -k 10 400 python tests/perf_handle.py > gpurun_out/perf_handle.json 2> gpurun_out/perf_handle.err || exit 1
echo "perf_handle ok"
for k in t j; do timeout -k 10 120 python tools/lone_k2t.py 16 --check --kind $k || exit 1; done
bash tools/gpurun/gpurun_hbm_sweep.sh
