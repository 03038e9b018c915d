#!/bin/bash
# round 5: kernel trace of C3 + AnchorLoopFast (is the loop GPU- or host-bound?)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05ar
mkdir -p $O
cd /tmp
echo "== rocprof C3 alf $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_alf -o run -- python3 $R/bench.py --config C3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3_alf.log 2>&1 || { tail -5 $O/prof_c3_alf.log; exit 1; }
tail -1 $O/prof_c3_alf.log | cut -c1-200
echo "== done $(date +%T)"
