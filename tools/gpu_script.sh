set -o pipefail
mkdir -p gpurun_out/sc
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_script_gpu.py tests/test_conseq_gpu.py tests/test_block_build_gpu.py tests/test_anchor_loop_gpu.py > gpurun_out/sc/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/sc/tests.log | tail -30
echo exit $rc
