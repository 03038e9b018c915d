#!/bin/bash
# round 5: the wide aligner's prefix word search -- parity (wide families, restarts, repeats,
# anchor loops), the wide batch bench, R3 + AnchorLoopFast; the switch off (NPGX_WIDE_LONG_HEAD=0) beside
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ag
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 1100 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py tests/test_anchor_loop_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lh in 128 0; do
  step "bench_wide lh$lh"
  NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide_$lh.log 2>&1 || { tail -5 $O/bench_wide_$lh.log; exit 1; }
  grep families $O/bench_wide_$lh.log | python -c "import sys, json; [print(d['families'], d['rows'], d['length'], d['unrelated_tails'], d['gpu_ms_batch'], d['speedup_vs_cpu_family_rate']) for d in map(json.loads, sys.stdin)]"
  step "r3 alf lh$lh"
  NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python bench.py --config R3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_R3_alf_$lh.log 2>&1 || { tail -5 $O/bench_R3_alf_$lh.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_R3_alf_$lh.log').read().strip().splitlines()[-1]); print('R3 alf', d['ms_per_step'], [(k['name'], round(k['ms'], 1)) for k in d.get('kernels_last_step', [])])"
done
step done
