#!/bin/bash
# round 5: the wide aligner's incremental head and first prefix after the
# prefix pass's early end (bench_wide), R3 + AnchorLoopFast at three heads, the
# C2 aligner's host phases (NPGX_PREP_DEBUG)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ak
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for v in 16:512 8:512 32:128 16:128 32:256; do
  lh=${v%%:*}; lm=${v#*:}
  step "bench_wide lh=$lh lm=$lm"
  NPGX_WIDE_LONG_HEAD=$lh NPGX_WIDE_LONG_M=$lm timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide_${lh}_$lm.log 2>&1 || { tail -5 $O/bench_wide_${lh}_$lm.log; exit 1; }
  python -c "
import json
for l in open('$O/bench_wide_${lh}_$lm.log'):
    if l.startswith('{'):
        d = json.loads(l); print($lh, $lm, d['families'], d['rows'], d['length'], d['gpu_ms_batch'], d['speedup_vs_cpu_family_rate'], d['checked_vs_oracle'])"
done
for lh in 128 32 16; do
  step "R3 alf lh=$lh"
  NPGX_WIDE_LONG_HEAD=$lh timeout -k 10 400 python bench.py --config R3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/r3_alf_$lh.log 2>&1 || { tail -5 $O/r3_alf_$lh.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/r3_alf_$lh.log').read().strip().splitlines()[-1]); print('R3 alf', $lh, d['ms_per_step'], d['value'])"
done
step "C2 prep"
NPGX_PREP_DEBUG=1 timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/c2_prep.log 2> $O/c2_prep.err || { tail -5 $O/c2_prep.err; exit 1; }
tail -1 $O/c2_prep.log | cut -c1-200
tail -25 $O/c2_prep.err
step done
