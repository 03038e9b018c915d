#!/bin/bash
# AnchorFinder parity (unit, sharded, full-size C2-C5) then the host phase times of a C3 step
set -o pipefail
mkdir -p gpurun_out/hd
TAG=${1:-af}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_anchor_finder_gpu.py \
    tests/test_af_sharded_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py tests/test_script_gpu.py \
    > gpurun_out/hd/tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/hd/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
NPGX_AF_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/hd/c3_$TAG.json 2> gpurun_out/hd/c3_$TAG.err
rc=$?; grep "af host" gpurun_out/hd/c3_$TAG.err | tail -2; cut -c1-200 gpurun_out/hd/c3_$TAG.json; exit $rc
