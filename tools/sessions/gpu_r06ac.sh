#!/bin/bash
# round 6: the device loop's final download reserves each block's fragment
# vectors: the loop's tests, smoke, C3 bench
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06ac
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_fullsize_gpu.py tests/test_anchor_loop_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2; do
  step "bench C3"
  timeout -k 10 300 python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_C3_$rep.log 2>&1 || { tail -5 $O/bench_C3_$rep.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C3_$rep.log').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], d['value'], d['stage_timeline']['ms']['elf_download'])"
done
step done
