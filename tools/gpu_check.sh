#!/bin/bash
# A focused GPU check (run via gpurun from the repo root):
#   tools/gpu_check.sh TAG "pytest -k expression or test files" [bench args...]
# runs the selected -m gpu tests, smoke, then one bench line with the given
# arguments (none: skip the bench).  Every GPU step has its own time limit and
# the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-chk}
TESTS=${2:-}
shift 2 || true
O=$R/gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ $# -gt 0 ]; then
  step bench
  timeout -k 10 600 python bench.py "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-400
fi
