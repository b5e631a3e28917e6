set -o pipefail
mkdir -p gpurun_out
EZ_K2=grp timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py > gpurun_out/gt_grp.log 2>&1
rc=$?; echo "pytest grp rc=$rc"; tail -3 gpurun_out/gt_grp.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp.sh
