#!/bin/bash
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04d
mkdir -p $O
echo "== ab twins C3 $(date +%T)"
tools/gpu_ab_env.sh r04d NPGX_TWINS 0 -1 --config C3 --steps 10 --warmup 3 || exit 1
for cfg in C3 C2 C4:pair; do
  echo "== hostprof $cfg $(date +%T)"
  timeout -k 10 300 python tools/host_profile.py $cfg 150 > $O/host_$cfg.txt 2>&1 || { tail -5 $O/host_$cfg.txt; exit 1; }
  head -30 $O/host_$cfg.txt
done
