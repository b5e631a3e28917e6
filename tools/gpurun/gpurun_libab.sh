set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/libab; rm -rf $O; mkdir -p $O
for L in ${LIBS:-libeazy_amd_s_max-ilp.so libeazy_amd.so libeazy_amd_s_max-memory-clause.so libeazy_amd_s_max-ilp.so libeazy_amd.so}; do
  EZ_LIB=$GRAFT_REPO_ROOT/eazy_amd/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 > $O/$L.json 2> $O/$L.err
  rc=$?; echo "$L rc=$rc $(python3 -c "import json;d=json.load(open('$O/$L.json'));print(round(d['value'],2),d['kernel_ms'])")"; [ $rc -eq 0 ] || exit $rc
done
