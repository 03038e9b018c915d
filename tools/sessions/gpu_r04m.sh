#!/bin/bash
# AnchorLoop (SplitExtendable, ExtendLoop, AddingLoopBySize) parity on the GPU
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04m
mkdir -p $O
echo "== pytest anchor loop $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_anchor_loop_full_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | cut -c1-200
