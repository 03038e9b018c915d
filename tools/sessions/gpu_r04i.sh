#!/bin/bash
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04i
mkdir -p $O
for cfg in rtiny rsmall; do
  echo "== diag_alf $cfg $(date +%T)"
  timeout -k 10 300 python tools/diag_alf.py $cfg > $O/diag_alf_$cfg.txt 2>&1 || { tail -30 $O/diag_alf_$cfg.txt; exit 1; }
  cat $O/diag_alf_$cfg.txt | cut -c1-200 | head -60
done
