#!/bin/bash
# round 6: split twins (NPGX_TWINS -1: launches with few tasks) at C3 / R3;
# two-row unsplit twins for the pair job
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06n
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for cfg in C3 R3; do
  step "split twins $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06n NPGX_TWINS 0 -1 --config $cfg --steps 10 --warmup 3 || exit 1
done
step "pairs utwins 2"
timeout -k 10 900 tools/gpu_ab_env.sh r06n NPGX_UTWINS 3 2 --mode pairs --config C4 --steps 2 --warmup 1 || exit 1
step done
