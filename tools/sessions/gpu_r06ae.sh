#!/bin/bash
# round 6: the unsplit twins' task cap (NPGX_UTWIN_TASKS 512, default, vs 768
# / 1024) at C3 and R3 on the final code
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
step() { echo "== $1 $(date +%T)"; }
for v in 768 1024; do
  for cfg in C3 R3; do
    step "NPGX_UTWIN_TASKS 512 vs $v, $cfg"
    timeout -k 10 600 tools/gpu_ab_env.sh r06ae NPGX_UTWIN_TASKS 512 $v --config $cfg --steps 10 --warmup 3 || exit 1
  done
done
step done
