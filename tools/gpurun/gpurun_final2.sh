#!/bin/bash
# Round-3 final measurement, part 2: C4, C4h, C4s (PMC traffic passes, bench lines with CPU baselines)
set -o pipefail
export TMPDIR=/tmp
WLS="c4 c4h c4s" bash gpurun_meas.sh
