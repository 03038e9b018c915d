#!/bin/bash
# Round-end evidence in one call: GPU tests, smoke, C3 bench (+cpu_baseline),
# rocprofv3 kernel stats of the bench, FETCH_SIZE / WRITE_SIZE passes (separate)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-final}
O=$R/gpurun_out/$TAG
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && exit $rc
cd /tmp
echo "== rocprof $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -3 $O/prof.log; exit $rc; }
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== $c $(date +%T)"
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/c3_$c -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_$c.log 2>&1 || { tail -5 $O/c3_$c.log; exit 1; }
done
echo "== done $(date +%T)"
