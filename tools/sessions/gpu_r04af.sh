#!/bin/bash
# AnchorLoop at C3: AddingLoopBySize round costs and a host sampling profile
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04af
mkdir -p $O
NPGX_AL_DEBUG=1 timeout -k 10 300 python bench.py --config C3 --anchor-loop full --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/bench_C3_al_dbg.log 2> $O/al_debug_C3.txt || { tail -5 $O/al_debug_C3.txt; exit 1; }
sort -t' ' -k2 -n -r $O/al_debug_C3.txt | grep "adding_loop" | sort -t, -k5 | tail -8
NPGX_PROFILE=1 timeout -k 10 300 python tools/host_profile.py C3 1 full > $O/host_C3_full.txt 2>&1 || { tail -5 $O/host_C3_full.txt; exit 1; }
head -32 $O/host_C3_full.txt
