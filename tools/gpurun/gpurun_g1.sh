set -o pipefail
mkdir -p gpurun_out
EZ_K1S_GIN=${GIN:-1} timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_stream.py > gpurun_out/gt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp.sh
