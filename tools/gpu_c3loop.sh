set -o pipefail
mkdir -p gpurun_out/c3l
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_loop_gpu.py tests/test_conseq_gpu.py tests/test_fullsize_c45_gpu.py -k "loop or conseq" > gpurun_out/c3l/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config C3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3l/c3_loop.json 2> gpurun_out/c3l/err.txt
rc=$?
tail -2 gpurun_out/c3l/tests.log
echo exit $rc
