set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/tail; rm -rf $O; mkdir -p $O
for N in 65536 131072 262144; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n$N -o run -- python3 bench.py --no-cpu --no-e2e --no-gather --steps 5 --warmup 1 --streams $N > $O/n$N.log 2>&1 || exit 1
  python3 - $O/n$N <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if any(k in n for k in ('k1_lean','k1_emit','k3_','k2_ring','k_edge','pad','copy')): print(sys.argv[1][-7:], n[:60], r['Calls'], round(float(r['AverageNs'])/1e6,4))
PY
done
