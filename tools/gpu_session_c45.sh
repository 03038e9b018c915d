set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_similar_aligner_gpu.py > gpurun_out/t_sa.log 2>&1 && \
timeout -k 10 300 $T tests/test_dp_gpu.py -k c5 > gpurun_out/t_dp.log 2>&1 && \
timeout -k 10 400 $T tests/test_fullsize_c45_gpu.py > gpurun_out/t_c45.log 2>&1 && \
timeout -k 10 300 $T tests/test_af_sharded_gpu.py -k "C4" > gpurun_out/t_shard.log 2>&1 && \
NPGX_SPLIT_DEBUG=1 timeout -k 10 300 python -u bench.py --config C4 --anchor-loop --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/b_c4loop.log 2>&1
echo exit $?
tail -3 gpurun_out/t_*.log
