#!/bin/bash
# PMC passes over one bench workload (one rocprofv3 run per counter set): bash gpurun_pmc.sh WORKLOAD "SET1" "SET2" ...
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc
rm -rf $O && mkdir -p $O
cd $GRAFT_REPO_ROOT
W=$1; shift
k=0
for C in "$@"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$k -o run -- python3 bench.py --no-cpu --no-e2e --no-gather --steps 2 --warmup 1 --workload $W > $O/p$k.log 2>&1 || { echo "pass $k failed"; tail -3 $O/p$k.log; exit 1; }
done
echo ok
