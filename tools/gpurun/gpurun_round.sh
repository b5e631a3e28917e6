#!/bin/bash
# Round measurement on one MI355X: GPU tests, kernel-trace profile, PMC traffic
# passes (their summary records the kernel-source hash, so bench.py can use it
# later from profiles/traffic_<workload>.json), then the bench line.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
rm -rf $O && mkdir -p $O
WL=${WL:-c1}
STREAMS=${STREAMS:-65536}
SB=${SB:-4096}
ARGS="--workload $WL ${BENCH_ARGS:-}"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 $ARGS > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run -- python3 bench.py --no-cpu --no-e2e --no-gather --steps 3 --warmup 1 $ARGS > $O/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py $O $O/traffic_$WL.json $WL $STREAMS $SB > $O/traffic.log 2>&1
timeout -k 10 600 python3 bench.py --traffic-json $O/traffic_$WL.json $ARGS > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
exit $rc
