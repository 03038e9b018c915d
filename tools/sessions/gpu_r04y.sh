#!/bin/bash
# host phases of the C3 step's start (AnchorFinder grouping, add_anchors,
# DummyAligner) and of the loop
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04y
mkdir -p $O
NPGX_AF_DEBUG=1 NPGX_BB_DEBUG=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench.log 2> $O/debug.txt || { tail -5 $O/debug.txt; exit 1; }
grep -E "af host|draft:" $O/debug.txt | tail -6
