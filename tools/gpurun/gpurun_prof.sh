cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/prof
rm -rf $O && mkdir -p $O
cd $GRAFT_REPO_ROOT
for w in ${WLS:-c4 c4h c4s}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w -o run -- python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workload $w > $O/$w.json 2> $O/$w.err || exit 1
done
