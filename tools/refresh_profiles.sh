#!/bin/bash
# Round-end evidence on the GPU box (run via gpurun from the repo root):
# full GPU test suite, smoke, C2 bench (+cpu_baseline), C3 bench, rocprofv3
# kernel stats of the C2 bench, PMC FETCH/WRITE passes, banded-DP bench.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench_c2
timeout -k 10 600 python bench.py > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-400
step bench_c3
timeout -k 10 600 python bench.py --config C3 --cpu-sample C3 --steps 5 --warmup 2 > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c1-300
step bench_c4
timeout -k 10 600 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-300
step timeline
timeout -k 10 300 python tools/align_timeline.py C2 > $O/align_timeline_c2.txt 2>&1 || { tail -5 $O/align_timeline_c2.txt; exit 1; }
step bench_dp
timeout -k 10 600 python tools/bench_dp.py > $O/bench_dp.log 2>&1 || { tail -5 $O/bench_dp.log; exit 1; }
tail -1 $O/bench_dp.log | cut -c1-300
step rocprof
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dp -o run -- python3 $R/tools/bench_dp.py --steps 2 --cpu-pairs 1 > $O/prof_dp.log 2>&1 || { tail -5 $O/prof_dp.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
step done
