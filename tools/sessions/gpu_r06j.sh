#!/bin/bash
# round 6: AnchorFinder Bloom epochs at C3 / C2 (0 = automatic)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06j
mkdir -p $O
echo "== sweep $(date +%T)"
NPGX_TIMERS=2 timeout -k 10 300 python tools/af_epoch_sweep.py C3,C2 0,4,8,12,16,24,32 6 > $O/sweep.txt 2>&1 || { tail -5 $O/sweep.txt; exit 1; }
cat $O/sweep.txt | cut -c1-160
echo "== done $(date +%T)"
