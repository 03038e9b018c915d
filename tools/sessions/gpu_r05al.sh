#!/bin/bash
# round 5: the wide aligner's shift-by-shift search with 3 barriers a shift
# (words kept in registers, the completing row raised in LDS): wide parity,
# the prefix pass over chunks of rows (NPGX_WIDE_PREFIX_CHUNK): bench_wide and
# R3 + AnchorLoopFast at heads 16 / 8 / 4, chunked or row by row
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05al
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py -k "wide" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_repeats_gpu.py > $O/pytest_rep.log 2>&1 || { tail -30 $O/pytest_rep.log; exit 1; }
tail -1 $O/pytest_rep.log
for v in 128:1 128:0 16:1 8:1 8:0 4:1; do
  lh=${v%%:*}; pc=${v#*:}
  step "bench_wide lh=$lh chunk=$pc"
  NPGX_WIDE_PREFIX_CHUNK=$pc NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide_${lh}_$pc.log 2>&1 || { tail -5 $O/bench_wide_${lh}_$pc.log; exit 1; }
  python -c "
import json
for l in open('$O/bench_wide_${lh}_$pc.log'):
    if l.startswith('{'):
        d = json.loads(l); print($lh, $pc, d['families'], d['rows'], d['length'], d['gpu_ms_batch'], d['speedup_vs_cpu_family_rate'], d['checked_vs_oracle'])"
done
for v in 16:1 8:1 8:0 4:1; do
  lh=${v%%:*}; pc=${v#*:}
  step "R3 alf lh=$lh chunk=$pc"
  NPGX_WIDE_PREFIX_CHUNK=$pc NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python bench.py --config R3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/r3_alf_${lh}_$pc.log 2>&1 || { tail -5 $O/r3_alf_${lh}_$pc.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/r3_alf_${lh}_$pc.log').read().strip().splitlines()[-1]); print('R3 alf', $lh, $pc, d['ms_per_step'], d['value'])"
done
step done
