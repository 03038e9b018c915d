#!/bin/bash
# round 5: A/B of the aligner's fast_run row batching (libnpge_amd_fr1.so = one row at a time, the
# round-4 order) and the prefix word search (NPGX_LONG_HEAD=0 = off), C3 and R3 bench lines
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05c
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for rep in 1 2; do
  for v in fr1:libnpge_amd_fr1.so next:libnpge_amd_next.so; do
    tag=${v%%:*}; lib=${v#*:}
    for cfg in C3 R3; do
      step "$tag $cfg rep $rep"
      NPGX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_${cfg}_$rep.log 2>&1 || { tail -5 $O/bench_${tag}_${cfg}_$rep.log; exit 1; }
      python -c "import json,sys; d=json.loads(open('$O/bench_${tag}_${cfg}_$rep.log').read().strip().splitlines()[-1]); print('$tag $cfg', d['ms_per_step'], d['last_step']['ms_stage']['align_batch'], d['last_step']['ms_stage']['anchor_finder'])"
    done
  done
done
step done
