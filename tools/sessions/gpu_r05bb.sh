#!/bin/bash
# round 5: AnchorLoop's failure path: the anchor-loop tests
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05bb
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_anchor_loop_full_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
echo "== done $(date +%T)"
