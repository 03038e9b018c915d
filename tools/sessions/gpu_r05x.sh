#!/bin/bash
# round 5: where C2's host time goes with the device loop (the aligner's batch preparation per
# iteration, SIGPROF samples of the library)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05x
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step prep_debug_c2
NPGX_PREP_DEBUG=1 timeout -k 10 300 python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/c2_prep.log 2> $O/c2_prep.err || { tail -5 $O/c2_prep.err; exit 1; }
grep "align_device" $O/c2_prep.err | tail -12
step hostprof_c2
timeout -k 10 300 python tools/host_profile.py C2 10 > $O/host_C2.txt 2>&1 || { tail -5 $O/host_C2.txt; exit 1; }
head -45 $O/host_C2.txt
step done
