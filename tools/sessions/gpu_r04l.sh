#!/bin/bash
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04l
mkdir -p $O
echo "== diag_alf rtiny $(date +%T)"
NPGX_ELF_DEBUG=1 ORACLE_ELF_DEBUG=1 timeout -k 10 300 python tools/diag_alf.py rtiny > $O/diag_alf_rtiny.txt 2>&1 || { tail -30 $O/diag_alf_rtiny.txt; exit 1; }
grep -v "^elf it" $O/diag_alf_rtiny.txt | cut -c1-200 | head -40
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_repeats_gpu.py tests/test_anchor_loop_gpu.py tests/test_block_build_gpu.py tests/test_align_pipe_gpu.py tests/test_fullsize_gpu.py tests/test_pairs_gpu.py tests/test_bench_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
