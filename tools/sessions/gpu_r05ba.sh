#!/bin/bash
# round 5: the wide aligner's switch point below 4 and a smaller first prefix (bench_wide, R3 + AnchorLoopFast)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ba
mkdir -p $O
for v in 4:512 2:512 4:256 1:512; do
  lh=${v%%:*}; lm=${v#*:}
  echo "== bench_wide lh=$lh lm=$lm $(date +%T)"
  NPGX_WIDE_LONG_HEAD=$lh NPGX_WIDE_LONG_M=$lm timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide_${lh}_$lm.log 2>&1 || { tail -5 $O/bench_wide_${lh}_$lm.log; exit 1; }
  python -c "
import json
for l in open('$O/bench_wide_${lh}_$lm.log'):
    if l.startswith('{'):
        d = json.loads(l); print($lh, $lm, d['families'], d['rows'], d['length'], d['gpu_ms_batch'], d['kernel_ms'], d['checked_vs_oracle'])"
  NPGX_WIDE_LONG_HEAD=$lh NPGX_WIDE_LONG_M=$lm timeout -k 10 400 python bench.py --config R3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/r3_alf_${lh}_$lm.log 2>&1 || { tail -5 $O/r3_alf_${lh}_$lm.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/r3_alf_${lh}_$lm.log').read().strip().splitlines()[-1]); print('R3 alf', $lh, $lm, d['ms_per_step'])"
done
echo "== done $(date +%T)"
