set -o pipefail
mkdir -p gpurun_out/fc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_build_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py tests/test_script_gpu.py -k "not anchor_finder" > gpurun_out/fc/tests.log 2>&1 && \
NPGX_FILTER_DEBUG=1 timeout -k 10 300 python -u bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/fc/c5.json 2> gpurun_out/fc/c5.err
rc=$?
tail -2 gpurun_out/fc/tests.log
grep "^filter" gpurun_out/fc/c5.err | tail -2
echo exit $rc
