#!/bin/bash
# repeat-rich parity incl. R3 at full size
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04ak
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_repeats_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | cut -c1-200
