set -o pipefail
mkdir -p gpurun_out/ou
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_build_gpu.py tests/test_anchor_loop_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py tests/test_script_gpu.py -k "not anchor_finder" > gpurun_out/ou/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config C3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ou/c3_loop.json 2> /dev/null && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ou/c3.json 2> /dev/null && \
timeout -k 10 300 python -u bench.py --config C2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ou/c2.json 2> /dev/null
rc=$?
tail -2 gpurun_out/ou/tests.log
echo exit $rc
