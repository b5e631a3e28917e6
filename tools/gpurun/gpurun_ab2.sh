#!/bin/bash
# GPU tests, then A/B of experiment libraries: K1L exchange visit (x0 vs x16384) and K2t round-start
# resolution with the 4-way search (x0 vs x8192) on C2 / C4s; handle Write latency x0 vs x16384
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/base $R/gpurun_out/ph
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/base/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/base/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="libeazy_amd_x0.so libeazy_amd_x8192.so libeazy_amd_x16384.so" WLS="c2 c4s" REPS=2 bash tools/gpurun/gpurun_lib_ab.sh || exit 1
for L in x0 x16384; do
  EZ_LIB=$R/eazy_amd/libeazy_amd_$L.so timeout -k 10 300 python3 tests/perf_handle.py --writes 1000 > $R/gpurun_out/ph/$L.json 2>&1 || { tail -5 $R/gpurun_out/ph/$L.json; exit 1; }
  python3 -c "import json;d=json.load(open('$R/gpurun_out/ph/$L.json'));print('$L', {k:round(v['gpu_us_p50'],1) for k,v in d.items() if isinstance(v,dict) and 'gpu_us_p50' in v})"
done
