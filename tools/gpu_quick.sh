# aligner + full-size parity, then the C3 and C4-loop benches (short)
set -o pipefail
mkdir -p gpurun_out/q
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_similar_aligner_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py tests/test_anchor_loop_gpu.py tests/test_block_build_gpu.py > gpurun_out/q/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/q/c3.json 2>gpurun_out/q/c3.err && \
timeout -k 10 300 python -u bench.py --config C4 --anchor-loop --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/q/c4loop.json 2>gpurun_out/q/c4loop.err
rc=$?
tail -3 gpurun_out/q/tests.log
echo exit $rc
