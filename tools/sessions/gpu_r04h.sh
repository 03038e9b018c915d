#!/bin/bash
# aligner phase cycles (the NPGX_SA_PROFILE build) on one C4 pair and on C3
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04h
mkdir -p $O
for cfg in C4:pair C3; do
  echo "== phases $cfg $(date +%T)"
  NPGX_PROFILE=1 timeout -k 10 300 python tools/analyze_bb.py $cfg > $O/phases_$cfg.txt 2>&1 || { tail -5 $O/phases_$cfg.txt; exit 1; }
  tail -25 $O/phases_$cfg.txt
done
