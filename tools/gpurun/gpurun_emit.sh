#!/bin/bash
# kernel averages of k1_emit with and without LDS staging
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/emit
rm -rf $O && mkdir -p $O
for V in 1 0; do
  EZ_K1E_STAGE=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$V -o run -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 > $O/p$V.log 2>&1
  rc=$?; echo "stage=$V rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -E "k1_emit|k1_parse|k3_gather|k2_ring" $O/p$V/run_kernel_stats.csv | cut -d, -f1,2,4 | sed 's/(.*)"/"/'
done
