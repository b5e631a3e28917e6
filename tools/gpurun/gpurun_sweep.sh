#!/bin/bash
# one gpurun call: GPU tests then a bench sweep over K1 variants (GS) and stream sizes (SZ)
set -o pipefail
mkdir -p gpurun_out
EZ_K1=${TK1:-} timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest=$rc"
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for G in ${GS:-lane g16 wave}; do
for Z in ${SZ:-4096}; do
  EZ_K1=$G timeout -k 10 300 python bench.py --no-cpu --steps 10 --stream-bytes $Z > gpurun_out/bench_G${G}_$Z.json 2> gpurun_out/bench_G${G}_$Z.err
  rc=$?
  echo "G=$G Z=$Z rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/bench_G${G}_$Z.json'));print(round(d['value'],2), {k:round(v,3) for k,v in d['kernel_ms'].items()}, round(d['compress_GiBps'],1), round(d['decompress_GiBps'],1))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done
done
