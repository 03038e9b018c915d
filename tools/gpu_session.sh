#!/bin/bash
# GPU session: parity tests, smoke, bench, rocprof kernel trace (run from repo root via gpurun)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-run}
mkdir -p gpurun_out
echo "== pytest gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
echo "== rocprof"; date
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-300; exit $rc
