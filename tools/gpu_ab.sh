#!/bin/bash
# DraftPangenome parity (block build, full-size C2/C3, sharded) then a C3 bench
set -o pipefail
mkdir -p gpurun_out/ab
TAG=${1:-ab}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_block_build_gpu.py tests/test_similar_aligner_gpu.py \
    tests/test_fullsize_gpu.py tests/test_af_sharded_gpu.py tests/test_anchor_loop_gpu.py > gpurun_out/ab/tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ab/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab/c3_$TAG.json 2> gpurun_out/ab/c3_$TAG.err
rc=$?; cut -c1-200 gpurun_out/ab/c3_$TAG.json
[ $rc -ne 0 ] && exit $rc
NPGX_FILTER_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/c3dbg_$TAG.json 2> gpurun_out/ab/c3dbg_$TAG.err
