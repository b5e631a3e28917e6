#!/bin/bash
# K2 routing data: every long-stream workload with the wave decoder (K2w) and the token-parallel one (K2t)
set -o pipefail
for W in ${WLS:-c2 c4 c4h c4s}; do
  BARGS="--no-check" STEPS=${STEPS:-3} bash tools/gpurun/gpurun_abq.sh $W EZ_K2=wave EZ_K2=tok || exit 1
done
