#!/bin/bash
# the aligner on R3 (repeat-rich): per-job costs and split statistics, for the next round
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04al
mkdir -p $O
NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py R3 > $O/analyze_R3.txt 2>&1 || { tail -5 $O/analyze_R3.txt; exit 1; }
head -60 $O/analyze_R3.txt | cut -c1-200
