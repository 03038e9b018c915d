#!/bin/bash
# host sampling profile of DraftPangenome -> AnchorLoop (C2), AnchorLoop parity at C2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04o
mkdir -p $O
echo "== hostprof C2 full $(date +%T)"
NPGX_PROFILE=1 timeout -k 10 300 python tools/host_profile.py C2 2 full > $O/host_C2_full.txt 2>&1 || { tail -5 $O/host_C2_full.txt; exit 1; }
head -45 $O/host_C2_full.txt
echo "== pytest anchor loop C2 $(date +%T)"
timeout -k 10 600 python -u -m pytest "tests/test_anchor_loop_full_gpu.py::test_anchor_loop[C2]" -m gpu -x -v --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | cut -c1-200
