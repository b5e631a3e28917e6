#!/bin/bash
# Round measurement on one MI355X, per workload: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
# -> tools/traffic.py (HBM bytes per launch, recorded with the kernel-source hash and shape), then the
# bench line with that traffic and its CPU baseline; for C1 also the kernel-trace profile.
#   WLS="c1 c2 c4" bash gpurun_meas.sh       (outputs: gpurun_out/meas/)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/meas
mkdir -p $O
declare -A SHAPE=([c1]="65536 4096" [c2]="4096 262144" [c3]="1048576 4096" [c4]="64 4194304" [c4h]="64 4194304" [c4s]="64 4194304")
for W in ${WLS:-c1}; do
  rm -rf $O/$W && mkdir -p $O/$W
  if [ "$W" = c1 ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$W/prof -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 --workload $W > $O/$W/prof.log 2>&1
    rc=$?; echo "$W prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  fi
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $O/$W/pmc_$C -o run -- python3 bench.py --no-cpu --no-e2e --no-gather --steps 2 --warmup 1 --workload $W > $O/$W/pmc_$C.log 2>&1
    rc=$?; echo "$W pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/traffic.py $O/$W $O/traffic_$W.json $W ${SHAPE[$W]} > $O/$W/traffic.log 2>&1 || { echo "$W traffic failed"; cat $O/$W/traffic.log; exit 1; }
  E=--no-e2e; [ "$W" = c1 ] && E=""
  timeout -k 10 600 python3 bench.py --traffic-json $O/traffic_$W.json --workload $W --steps ${STEPS:-10} $E > $O/$W.json 2> $O/$W.err
  rc=$?; echo "$W bench rc=$rc $(python3 -c "import json;d=json.load(open('$O/$W.json'));c=d.get('cpu_baseline') or {};r=d['roofline'];print(round(d['value'],2), {k:round(v,3) for k,v in d['kernel_ms'].items()}, 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'cpu', c.get('value'), c.get('single_thread',{}).get('value'))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || { tail -5 $O/$W.err; exit $rc; }
done
