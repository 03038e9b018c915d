#!/bin/bash
# round 6: the aligner's waves a SIMD chosen per launch (4 past 2048 tasks,
# else 2): the whole GPU suite, then C5 / C3 / C2 / R3 benches
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06u
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest gpu"
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in C5 C3 C2 R3 C5 C3; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['value'], {k: v for k, v in d['stage_timeline']['ms'].items() if v > 0.5})"
done
step done
