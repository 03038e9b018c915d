#!/bin/bash
# round 6: OverlaplessUnion's priority order by a radix sort of packed
# leading fields with the ties put in order by the full comparator
# (k_ou_runs) instead of the comparator merge sort (libnpge_amd_alt.so), v2
# packed key (size 8 bits, length 24, start 32); and goodSlices' frame test
# of every window start as device bits (k_fi_wbits; alt: the host slides the
# frame sum): parity, A/B at C3 / C2 / C5 (the stage timeline separates them:
# OverlaplessUnion vs Filter)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06z2
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_block_build_gpu.py tests/test_fullsize_gpu.py tests/test_anchor_device_gpu.py tests/test_repeats_gpu.py tests/test_fullsize_c45_gpu.py tests/test_align_pipe_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C2 C5; do
  step "radix OU order (new) vs merge sort (alt), $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config $cfg --steps 10 --no-pairs-line > $O/ab_ou_radix_$cfg.txt 2>&1 || { tail -5 $O/ab_ou_radix_$cfg.txt; exit 1; }
  cut -c1-170 $O/ab_ou_radix_$cfg.txt
done
step done
