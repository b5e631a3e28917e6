# bench.py with 1..4 batches in flight per workload (WLS, INF): value, step time, per-launch event times
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/inf; rm -rf $O; mkdir -p $O
for W in ${WLS:-c1 c2 c4 c4h c4s}; do
  for I in ${INF:-1 2}; do
    timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 8 --warmup 4 --workload $W --inflight $I > $O/${W}_$I.json 2> $O/${W}_$I.err || { tail -5 $O/${W}_$I.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${W}_$I.json'));print('$W', $I, round(d['value'],2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_ms'].items()}, d.get('kernel_ms_isolated') and {k:round(v,3) for k,v in d['kernel_ms_isolated'].items()})"
  done
done
