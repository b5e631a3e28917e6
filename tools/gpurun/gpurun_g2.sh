set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/ps
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ps -o run -- python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1 > gpurun_out/ps.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/ps -name "*kernel_stats.csv" | head -1 | xargs cat | grep "ez::" | cut -d, -f1-4
