#!/bin/bash
# round 5: the buffer cache's own test and the allocation-path GPU tests with the cache off (default)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aw
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_buf_cache_gpu.py tests/test_elf_device_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "== done $(date +%T)"
