set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_fullsize_c45_gpu.py -k "draft" > gpurun_out/c5/tests.log 2>&1
rc=$?
tail -6 gpurun_out/c5/tests.log
echo exit $rc
