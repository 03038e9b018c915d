#!/bin/bash
# round 5: the wide aligner's prefix pass ends at the first row that raises no
# word: wide parity, then tools/bench_wide.py at incremental heads 128 / 64 / 32
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aj
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py -k "wide" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_repeats_gpu.py > $O/pytest_rep.log 2>&1 || { tail -30 $O/pytest_rep.log; exit 1; }
tail -1 $O/pytest_rep.log
for lh in 128 64 32; do
  step "bench_wide lh=$lh"
  NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide_$lh.log 2>&1 || { tail -5 $O/bench_wide_$lh.log; exit 1; }
  python -c "
import json
for l in open('$O/bench_wide_$lh.log'):
    if l.startswith('{'):
        d = json.loads(l); print($lh, d['families'], d['rows'], d['length'], d['gpu_ms_batch'], d['speedup_vs_cpu_family_rate'], d['checked_vs_oracle'])"
done
step done
