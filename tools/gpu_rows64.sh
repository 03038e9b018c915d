set -o pipefail
mkdir -p gpurun_out/r64
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_anchor_loop_gpu.py -k "64" > gpurun_out/r64/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r64/tests.log | tail -8
echo exit $rc
