#!/bin/bash
# ExtendLoopFast's first-lap hashing overlapped with the flank alignment:
# parity (block build, full size, pairs, anchor loops, repeats), then A/B of
# the C3 line and the pairs line on this box (NPGX_ELF_NO_OVERLAP=1: hash first)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04aa
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_block_build_gpu.py tests/test_fullsize_gpu.py tests/test_pairs_gpu.py tests/test_anchor_loop_gpu.py tests/test_anchor_loop_full_gpu.py tests/test_repeats_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
for ab in 0 1 0 1; do
  if [ $ab = 1 ]; then export NPGX_ELF_NO_OVERLAP=1; else unset NPGX_ELF_NO_OVERLAP; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_C3_$ab.log 2>&1 || { tail -5 $O/bench_C3_$ab.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C3_$ab.log').read().strip().splitlines()[-1]); print('C3 no_overlap=$ab', d['value'], d['ms_per_step'])"
done
for ab in 0 1; do
  if [ $ab = 1 ]; then export NPGX_ELF_NO_OVERLAP=1; else unset NPGX_ELF_NO_OVERLAP; fi
  timeout -k 10 300 python bench.py --mode pairs --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$ab.log 2>&1 || { tail -5 $O/pairs_$ab.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$ab.log').read().strip().splitlines()[-1]); print('pairs no_overlap=$ab', d['value'], d['ms_per_step'])"
done
