#!/bin/bash
# GPU session script (run via gpurun from the repo root)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
echo "== pytest gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"; date
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
echo "== rocprof"; date
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
rc=$?; tail -3 $R/gpurun_out/prof.log; exit $rc
