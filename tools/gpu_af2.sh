set -o pipefail
mkdir -p gpurun_out/af2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py -k "anchor_finder or sharded" > gpurun_out/af2/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/af2/c3.json 2>/dev/null && \
timeout -k 10 300 python -u bench.py --config C4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/af2/c4.json 2>/dev/null
rc=$?
tail -2 gpurun_out/af2/tests.log
echo exit $rc
