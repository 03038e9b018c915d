#!/bin/bash
# round 6: where the C3 aligner time goes now: the profiling build's phase
# counters (host loop: job statistics), a kernel trace of the default C3 line
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06b
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "analyze prof C3"
NPGX_ELF_DEVICE=0 NPGX_PROFILE=1 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_C3_prof.txt 2>&1 || { tail -5 $O/analyze_C3_prof.txt; exit 1; }
grep -E "phase cycles|fit cycles|cycles per column" $O/analyze_C3_prof.txt
step "analyze C3 (timeline)"
NPGX_ELF_DEVICE=0 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_C3.txt 2>&1 || { tail -5 $O/analyze_C3.txt; exit 1; }
mv gpurun_out/jobstats_C3.npy $O/ || true
mv gpurun_out/jobstats_C3_prof.npy $O/ || true
step rocprof_c3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
python3 $R/tools/step_timeline.py $O/prof_c3/run_kernel_trace.csv > $O/c3_step_timeline.txt 2>&1 || true
head -5 $O/c3_step_timeline.txt
step done
