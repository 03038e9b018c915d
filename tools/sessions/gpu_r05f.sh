#!/bin/bash
# round 5: which table pass breaks in the count / scan / fill form (each alone, then all)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05f
mkdir -p $O
echo "== pytest_multi $(date +%T)"
NPGX_ELF_SYNC=1 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_elf_device_gpu.py -k multi_launch > $O/pytest_multi.log 2>&1
rc=$?
grep -E "PASSED|FAILED|elf check|Error" $O/pytest_multi.log | cut -c1-600 | head -40
exit $rc
