#!/bin/bash
# SQ counters (3 passes) and one TA/TD/TCP pass over the C1 bench at the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
SQ_KERNELS="k1_lean k2_ring k1_emit" bash tools/gpurun/gpurun_sq.sh --workload c1 || exit 1
O=$R/gpurun_out/ta; rm -rf $O; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 bench.py --no-cpu --no-e2e --no-gather --steps 2 --warmup 1 --workload c1 > $O/p1.log 2>&1
rc=$?; echo "ta pass rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p1.log; exit $rc; }
python3 tools/pmc_sum.py $O/p1/run_counter_collection.csv k1_lean k2_ring k1_emit
