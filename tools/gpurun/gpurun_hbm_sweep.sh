#!/bin/bash
# BASELINE config 3 ("rocprof HBM GB/s vs roofline sweep"): log-like batches of 1 GiB cut into
# streams of 4 KiB .. 1 MiB (block 1 MiB, htable 1024).  Per size: the bench line (kernel times,
# routing), then FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 --pmc runs) for the
# per-kernel HBM bytes; tools/hbm_sweep.py joins them into one table.
#   bash tools/gpurun/gpurun_hbm_sweep.sh            (sizes: SZ="4096 16384 65536 262144 1048576")
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sweep
rm -rf $O && mkdir -p $O
TOTAL=$((1 << 30))
for Z in ${SZ:-4096 16384 65536 262144 1048576}; do
  N=$((TOTAL / Z))
  A="--workload c2 --stream-bytes $Z --streams $N --no-e2e --no-cpu --inflight 1"  # (per-kernel times: one batch at a time)
  timeout -k 10 300 python3 bench.py $A --steps 5 --warmup 1 > $O/b_$Z.json 2> $O/b_$Z.err
  rc=$?; echo "size $Z bench rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/b_$Z.err; exit $rc; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/p_$Z/pmc_$C -o run -- python3 bench.py $A --no-gather --steps 2 --warmup 1 > $O/p_${Z}_$C.log 2>&1
    rc=$?; echo "size $Z pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/traffic.py $O/p_$Z $O/t_$Z.json c2 $N $Z > /dev/null 2>&1 || exit 1
done
python3 tools/hbm_sweep.py $O ${SZ:-4096 16384 65536 262144 1048576} | tee $O/sweep.txt
