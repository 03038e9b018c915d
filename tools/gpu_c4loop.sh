# C4 DraftPangenome -> AnchorLoopFast: parity vs the fixture, then bench steps (stage split in last_step.anchor_loop)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_c45_gpu.py -k anchor_loop > gpurun_out/t_c4loop.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config C4 --anchor-loop --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_c4loop.log 2>&1
echo exit $?
