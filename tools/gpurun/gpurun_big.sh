#!/bin/bash
# C1-shaped run past the Infinity Cache (262,144 x 4 KiB = 1 GiB of input): PMC FETCH_SIZE / WRITE_SIZE
# passes and the traffic summary (gpurun_out/big/traffic_c1_1g.json), to tell HBM bytes from IC hits
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/big
rm -rf $O && mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run -- python3 bench.py --no-cpu --no-e2e --steps 2 --warmup 1 --streams 262144 > $O/pmc_$C.log 2>&1
  rc=$?; echo "big pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py $O $O/traffic_c1_1g.json c1 262144 4096 > $O/traffic.log 2>&1 || { cat $O/traffic.log; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 10 --streams 262144 --traffic-json $O/traffic_c1_1g.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "big bench rc=$rc"; exit $rc
