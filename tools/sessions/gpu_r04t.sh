#!/bin/bash
# AnchorLoop: AddingLoopBySize round costs (C2)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04t
mkdir -p $O
NPGX_AL_DEBUG=1 timeout -k 10 400 python bench.py --config C2 --anchor-loop full --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/bench_C2.log 2> $O/al_debug_C2.txt || { tail -5 $O/al_debug_C2.txt; exit 1; }
sort -t, -k1 $O/al_debug_C2.txt | awk '{print}' | head -80
