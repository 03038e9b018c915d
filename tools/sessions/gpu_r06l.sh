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
step done
