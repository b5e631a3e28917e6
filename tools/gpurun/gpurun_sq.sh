#!/bin/bash
# SQ counter passes over the C1 bench (one rocprofv3 --pmc run per pass): bash tools/gpurun/gpurun_sq.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=$R/gpurun_out/${SQ_OUT:-sq}; rm -rf $O; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
P3="SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS"
k=0
for P in "$P1" "$P2" "$P3"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$k -o run -- python3 bench.py --no-cpu --no-e2e --no-gather --steps 2 --warmup 1 $* > $O/p$k.log 2>&1
  rc=$?; echo "pass $k rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p$k.log; exit $rc; }
done
python3 tools/pmc_sum.py $O/p*/run_counter_collection.csv ${SQ_KERNELS:-k1_lean k2_ring k1_emit} > $O/sum.txt; cat $O/sum.txt
