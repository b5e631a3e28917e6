#!/bin/bash
# one gpurun call: GPU tests (default config) then a bench sweep over K1 group sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
echo "pytest=$?"
tail -5 gpurun_out/gpu_tests.log
for G in ${GS:-16 32 64}; do
  EZ_K1_G=$G timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/bench_G$G.json 2> gpurun_out/bench_G$G.err
  echo "G=$G rc=$? $(python -c "import json;d=json.load(open('gpurun_out/bench_G$G.json'));print(round(d['value'],2), d['kernel_ms'], round(d['compress_GiBps'],1), round(d['decompress_GiBps'],1))" 2>&1 | tail -1)"
done
