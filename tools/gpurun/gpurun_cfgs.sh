#!/bin/bash
# every non-C1 workload's bench line with its CPU baseline (bounded sample), one GPU
O=$GRAFT_REPO_ROOT/gpurun_out/cfg
rm -rf $O && mkdir -p $O
for w in ${WLS:-c2 c3 c4 c4h c4s}; do
  timeout -k 10 400 python3 bench.py --no-e2e --steps ${STEPS:-5} --warmup 1 --workload $w > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -3 $O/$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$w.json'));c=d.get('cpu_baseline') or {};print('$w', round(d['value'],2), {k:round(v,3) for k,v in d['kernel_ms'].items()}, 'cpu', c.get('value'), c.get('compress_GiBps'), c.get('decompress_GiBps'))"
done
