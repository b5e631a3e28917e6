set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc2; mkdir -p $R/gpurun_out/pmc2
for PAD in 0 8192; do
  EZ_K1S_LDSPAD=$PAD timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum,TCC_MISS_sum,TCP_TCC_READ_REQ_sum,TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $R/gpurun_out/pmc2/pad$PAD -o run -- python3 bench.py --no-cpu --no-e2e --steps 2 --warmup 1 > $R/gpurun_out/pmc2/pad$PAD.log 2>&1 || exit 1
  echo "pad $PAD ok"
done
timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --steps 5 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernel_ms'])"
