#!/bin/bash
# PMC passes (one counter group per pass, no tracing domains mixed in)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1 || true
i=0
for C in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 ${BENCH_ARGS:-} > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $C"
  [ $rc -ne 0 ] && tail -5 $R/gpurun_out/pmc/p$i.log && exit $rc
done
exit 0
