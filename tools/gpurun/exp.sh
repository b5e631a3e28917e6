#!/bin/bash
# experiment sweep: each line "ENV... -- bench args"; prints kernel ms per line
set -o pipefail
mkdir -p gpurun_out/exp
n=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  n=$((n+1))
  envs="${line%%--*}"; args="${line#*--}"
  env $envs timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 $args > gpurun_out/exp/e$n.json 2> gpurun_out/exp/e$n.err
  rc=$?
  echo "[$line] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/exp/e$n.json'));print(round(d['value'],2), {k:round(v,3) for k,v in d['kernel_ms'].items()}, round(d['ratio'],3))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done < "${1:-tools/exp.txt}"
