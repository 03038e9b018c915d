#!/bin/bash
# round 5: split segment length and long-job deferral thresholds with the prefix search (C3, C5)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05s
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for v in s256:256:500 s384:384:500 s512:512:500 d250:384:250 d1000:384:1000; do
  IFS=: read tag sp df <<< "$v"
  for cfg in C3 C5; do
    step "$tag $cfg"
    NPGX_ALIGN_SPLIT=$sp NPGX_ALIGN_DEFER=$df timeout -k 10 300 python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_$cfg.log 2>&1 || { tail -5 $O/bench_${tag}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${tag}_$cfg.log').read().strip().splitlines()[-1]); print('$tag $cfg', d['ms_per_step'])"
  done
done
step done
step "c3 critical paths"
NPGX_ELF_DEVICE=0 NPGX_SPLIT_DEBUG=1 NPGX_JOB_STATS=1 timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/c3_paths.log 2> $O/c3_paths.err || { tail -5 $O/c3_paths.err; exit 1; }
grep -E "^launch|^sub launch|^subs " $O/c3_paths.err | tail -40
step done2
