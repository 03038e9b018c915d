#!/bin/bash
# round 6: unsplit twins within 1024 tasks; the prefix search's LDS table:
# C3 kernel trace, k_align_jobs FETCH / WRITE per launch with and without it
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06f
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "ab utwins C3"
timeout -k 10 600 tools/gpu_ab_env.sh r06f NPGX_UTWINS 0 3 --config C3 --steps 10 --warmup 3 || exit 1
cd /tmp
step "rocprof C3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
for ll in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    step "pmc $c long_lds $ll"
    NPGX_LONG_LDS=$ll timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/c3_${c}_ll$ll -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/pmc_${c}_ll$ll.log 2>&1 || { tail -5 $O/pmc_${c}_ll$ll.log; exit 1; }
  done
done
step done
