#!/bin/bash
# round 5: the wide aligner at its new defaults (prefix search after 4
# shift-by-shift steps, 3 barriers a step, the prefix pass ending at a row that
# raises no word): aligner / repeat / anchor-loop parity, bench_wide, R3 lines
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05am
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py tests/test_anchor_loop_full_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step bench_wide
timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide.log 2>&1 || { tail -5 $O/bench_wide.log; exit 1; }
grep '^{' $O/bench_wide.log | cut -c1-260
for m in "R3:" "R3:--anchor-loop"; do
  cfg=${m%%:*}; fl=${m#*:}; tag=$cfg${fl:+_alf}
  step "bench $tag"
  timeout -k 10 400 python bench.py --config $cfg $fl --steps 5 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['value'])"
done
step done
