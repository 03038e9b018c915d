#!/bin/bash
# Round-end evidence on the GPU box (run via gpurun from the repo root), in
# two parts that each fit one gpurun call:
#   tools/round_end.sh TAG tests   -- full GPU suite, smoke, the default bench
#                                    (C3 with cpu_baseline, the driver's line)
#   tools/round_end.sh TAG perf    -- C2/C4/C5/anchor-loop benches, a C3 kernel
#                                    trace + stats, PMC FETCH_SIZE / WRITE_SIZE
#                                    passes (separate runs), the banded-DP bench
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-r03}
PART=${2:-tests}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ "$PART" = tests ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  step bench_c3
  timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
  tail -1 $O/bench_c3.log | cut -c1-300
else
  for cfg in C2 C4 C5 R3; do
    step bench_$cfg
    timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
    tail -1 $O/bench_$cfg.log | cut -c1-200
  done
  for cfg in C3 C4; do
    step bench_${cfg}_alf
    timeout -k 10 300 python bench.py --config $cfg --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_alf.log 2>&1 || { tail -5 $O/bench_${cfg}_alf.log; exit 1; }
    tail -1 $O/bench_${cfg}_alf.log | cut -c1-200
  done
  step bench_dp
  timeout -k 10 300 python tools/bench_dp.py > $O/bench_dp.log 2>&1 || { tail -5 $O/bench_dp.log; exit 1; }
  step rocprof_c3
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
  python3 $R/tools/step_timeline.py $O/prof_c3/run_kernel_trace.csv > $O/c3_step_timeline.txt 2>&1 || true
  step rocprof_c2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
  python3 $R/tools/step_timeline.py $O/prof_c2/run_kernel_trace.csv > $O/c2_step_timeline.txt 2>&1 || true
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_$c
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/c3_$c -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
  done
  cd $R
  step bench_pairs
  timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_pairs.log 2>&1 || { tail -5 $O/bench_pairs.log; exit 1; }
  tail -1 $O/bench_pairs.log | cut -c1-200
  cd /tmp
  step rocprof_pairs
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pairs -o run -- python3 $R/bench.py --mode pairs --config C4 --pairs 32 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_pairs.log 2>&1 || { tail -5 $O/prof_pairs.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_pairs_$c
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pairs_$c -o run -- python3 $R/bench.py --mode pairs --config C4 --pairs 32 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_pairs_$c.log 2>&1 || { tail -5 $O/pmc_pairs_$c.log; exit 1; }
  done
fi
step done
