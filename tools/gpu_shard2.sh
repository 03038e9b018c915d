set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_af_sharded_gpu.py -k "anchor_loop or draft" > gpurun_out/s2/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/s2/tests.log | tail -10
echo exit $rc
