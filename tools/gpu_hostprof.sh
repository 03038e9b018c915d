#!/bin/bash
# Host-side evidence of the block build (run via gpurun from the repo root):
# SIGPROF samples of the library during DraftPangenome steps (C3, C2, one C4
# pair), then a rocprofv3 kernel trace of a 3-step C3 bench with the step's
# GPU idle gaps.  Usage: tools/gpu_hostprof.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-hp}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for cfg in C3 C2 C4:pair; do
  step hostprof_$cfg
  timeout -k 10 300 python tools/host_profile.py $cfg 10 > $O/host_$cfg.txt 2>&1 || { tail -5 $O/host_$cfg.txt; exit 1; }
  head -40 $O/host_$cfg.txt
done
step split_debug_c3
NPGX_SPLIT_DEBUG=1 NPGX_JOB_STATS=1 NPGX_PREP_DEBUG=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/split_debug_c3.txt 2>&1 || { tail -5 $O/split_debug_c3.txt; exit 1; }
step align_timeline_c3
timeout -k 10 300 python tools/align_timeline.py C3 > $O/align_timeline_c3.txt 2>&1 || { tail -5 $O/align_timeline_c3.txt; exit 1; }
step analyze_c3
timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_c3.txt 2>&1 || { tail -5 $O/analyze_c3.txt; exit 1; }
step rocprof_c3
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
python tools/step_timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/c3_step_timeline.txt 2>&1
head -12 $O/c3_step_timeline.txt
step done
