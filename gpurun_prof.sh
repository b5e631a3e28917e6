#!/bin/bash
# kernel-trace + stats profile of bench.py (args passed through) into gpurun_out/prof_$TAG
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
mkdir -p $R/gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 bench.py "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "prof $TAG rc=$rc"
f=$(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(r['Name'][:60].ljust(60), r['Calls'], 'avg_ms=%.4f' % (float(r['AverageNs'])/1e6), 'pct=%s' % r['Percentage'])
"
exit $rc
