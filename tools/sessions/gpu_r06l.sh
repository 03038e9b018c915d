#!/bin/bash
# round 6: the aligner's split segment length and defer threshold at C3 / R3
# with this round's kernels (twins, 2 waves per SIMD, batched chain copies)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06l
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for cfg in C3 R3; do
  step "split $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06l NPGX_ALIGN_SPLIT 384 256 --config $cfg --steps 10 --warmup 3 || exit 1
  timeout -k 10 600 tools/gpu_ab_env.sh r06l NPGX_ALIGN_SPLIT 384 512 --config $cfg --steps 10 --warmup 3 || exit 1
  step "defer $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06l NPGX_ALIGN_DEFER 500 300 --config $cfg --steps 10 --warmup 3 || exit 1
  timeout -k 10 600 tools/gpu_ab_env.sh r06l NPGX_ALIGN_DEFER 500 800 --config $cfg --steps 10 --warmup 3 || exit 1
  step "utwin tasks $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06l NPGX_UTWIN_TASKS 512 768 --config $cfg --steps 10 --warmup 3 || exit 1
done
step "split waves 8: parity"
NPGX_LIB=libnpge_amd_sw8.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_fullsize_gpu.py > $O/pytest_sw8.log 2>&1 || { tail -30 $O/pytest_sw8.log; exit 1; }
tail -1 $O/pytest_sw8.log
for cfg in C3 R3; do
  step "split waves 8: ab $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_sw8.so 2 --config $cfg --no-pairs-line > $O/ab_sw8_$cfg.txt 2>&1 || { tail -5 $O/ab_sw8_$cfg.txt; exit 1; }
  cut -c1-150 $O/ab_sw8_$cfg.txt
done
step done
