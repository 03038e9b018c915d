#!/bin/bash
# round 5: DeConSeq compacts an arena of mostly dead rows on the device before
# downloading it: AnchorLoop parity, then C3 / C4 / R3 + AnchorLoopFast with and
# without (NPGX_DECONSEQ_NO_COMPACT=1)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ao
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_loop_full_gpu.py tests/test_repeats_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C4 R3; do
  for v in on off; do
    step "$cfg alf $v"
    if [ $v = off ]; then export NPGX_DECONSEQ_NO_COMPACT=1; else unset NPGX_DECONSEQ_NO_COMPACT; fi
    timeout -k 10 400 python bench.py --config $cfg --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/${cfg}_alf_$v.log 2>&1 || { tail -5 $O/${cfg}_alf_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/${cfg}_alf_$v.log').read().strip().splitlines()[-1]); a=d['last_step']['anchor_loop']; print('$cfg $v', d['ms_per_step'], 'deconseq', round(a['ms_loop']['deconseq'], 2))"
  done
done
unset NPGX_DECONSEQ_NO_COMPACT
step done
