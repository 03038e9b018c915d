set -o pipefail
mkdir -p gpurun_out/lc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_build_gpu.py tests/test_anchor_loop_gpu.py tests/test_conseq_gpu.py tests/test_script_gpu.py tests/test_fullsize_c45_gpu.py -k "not anchor_finder_c45" > gpurun_out/lc/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config C4 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lc/C4_loop.json 2> gpurun_out/lc/C4_loop.err
rc=$?
tail -2 gpurun_out/lc/tests.log
echo exit $rc
