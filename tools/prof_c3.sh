#!/bin/bash
# Quick C3 evidence on the GPU box (run via gpurun from the repo root): the C3
# bench line (no CPU baseline), the aligner's per-launch timeline, and a
# rocprofv3 kernel summary of a 3-step bench.  Usage: tools/prof_c3.sh TAG [CONFIG]
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-r03}
CFG=${2:-C3}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step bench
timeout -k 10 600 python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
step timeline
timeout -k 10 300 python tools/align_timeline.py $CFG > $O/align_timeline.txt 2>&1 || { tail -5 $O/align_timeline.txt; exit 1; }
step rocprof
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
step done
