set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_af_sharded_gpu.py tests/test_anchor_finder_gpu.py tests/test_fullsize_gpu.py -k "sharded or anchor_finder" > gpurun_out/s/tests.log 2>&1
rc=$?
tail -8 gpurun_out/s/tests.log
echo exit $rc
