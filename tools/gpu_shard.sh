set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_af_sharded_gpu.py > gpurun_out/s/tests.log 2>&1
rc=$?
tail -15 gpurun_out/s/tests.log
echo exit $rc
