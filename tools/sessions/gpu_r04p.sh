#!/bin/bash
# AnchorFinder at C5: kernel split per Bloom epoch count
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04p
mkdir -p $O
echo "== af epochs C5 $(date +%T)"
NPGX_TIMERS=2 timeout -k 10 400 python tools/af_epoch_sweep.py C5 1,2,4,8,0 3 > $O/af_epochs_c5.txt 2>&1 || { tail -5 $O/af_epochs_c5.txt; exit 1; }
cat $O/af_epochs_c5.txt
