#!/bin/bash
# round-5 baseline: C3 and R3 aligner per-job costs (plain and phase-profiled builds)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05a
mkdir -p $O
NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_C3.txt 2>&1 || { tail -5 $O/analyze_C3.txt; exit 1; }
NPGX_PROFILE=1 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_C3_prof.txt 2>&1 || { tail -5 $O/analyze_C3_prof.txt; exit 1; }
NPGX_PROFILE=1 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py R3 > $O/analyze_R3_prof.txt 2>&1 || { tail -5 $O/analyze_R3_prof.txt; exit 1; }
head -40 $O/analyze_C3_prof.txt | cut -c1-300
