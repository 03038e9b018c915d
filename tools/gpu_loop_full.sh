set -o pipefail
mkdir -p gpurun_out/lf
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_c45_gpu.py -k "anchor_loop" > gpurun_out/lf/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/lf/tests.log | tail -6
echo exit $rc
