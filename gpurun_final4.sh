#!/bin/bash
# Round-3 final measurement at the final sources: C1, C2, C4, C4h, C4s (MEAS overrides)
set -o pipefail
export TMPDIR=/tmp
WLS="${MEAS:-c1 c2}" bash gpurun_meas.sh
