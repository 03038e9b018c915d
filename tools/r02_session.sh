#!/bin/bash
# Round-2 GPU session (run from the repo root via gpurun): GPU tests, smoke,
# the default bench (C3 + cpu_baseline), rocprofv3 kernel stats of the C3
# bench, PMC FETCH/WRITE passes at C3.  usage: r02_session.sh TAG [quick]
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-r02}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench_c3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
cut -c1-600 $O/bench_c3.json
step bench_c2
timeout -k 10 600 python bench.py --config C2 --steps 20 --warmup 5 --cpu-runs 3 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-300 $O/bench_c2.json
step bench_c3_loop
timeout -k 10 600 python bench.py --anchor-loop --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c3_loop.json 2> $O/bench_c3_loop.err || { tail -5 $O/bench_c3_loop.err; exit 1; }
cut -c1-300 $O/bench_c3_loop.json
step bench_c4
timeout -k 10 600 python bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
cut -c1-300 $O/bench_c4.json
[ "$2" = quick ] && { step done; exit 0; }
step rocprof_c3
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/c3_$c -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_$c.log 2>&1 || { tail -5 $O/c3_$c.log; exit 1; }
done
step done
