#!/bin/bash
# wide (> 64 rows) aligner parity on the GPU, then the rest of the aligner tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-wide}
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    tests/test_similar_aligner_gpu.py -k "more_than_64" > gpurun_out/wide_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/wide_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    tests/test_anchor_loop_gpu.py -k "more_than_64 or more_than_64_fragments" >> gpurun_out/wide_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/wide_$TAG.log; exit $rc
