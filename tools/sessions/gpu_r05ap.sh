#!/bin/bash
# round 5: C3 + AnchorLoopFast with the wide aligner's old switch point (128)
# against the new one (4), alternating on one box
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ap
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for v in 4a 128a 4b 128b; do
  lh=${v%[ab]}
  step "C3 alf lh=$lh ($v)"
  NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python bench.py --config C3 --anchor-loop --steps 5 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/C3_alf_$v.log 2>&1 || { tail -5 $O/C3_alf_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/C3_alf_$v.log').read().strip().splitlines()[-1]); a=d['last_step']['anchor_loop']; print('$v', d['ms_per_step'], {k: round(x, 1) for k, x in a['ms_loop'].items()})"
done
step done
