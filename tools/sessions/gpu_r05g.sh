#!/bin/bash
# round 5: the device loop's C3 step against the host loop's (kernel traces + stats, step timelines),
# and the prefix word search on / off (NPGX_LONG_HEAD=0) at C3 / R3
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05g
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for v in host:0 dev:1; do
  IFS=: read tag dev <<< "$v"
  step "rocprof $tag"
  cd /tmp
  NPGX_ELF_DEVICE=$dev timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_$tag.log 2>&1 || { tail -5 $O/prof_$tag.log; exit 1; }
  cd $R
  f=$(ls $O/prof_$tag/*/run_kernel_trace.csv $O/prof_$tag/run_kernel_trace.csv 2>/dev/null | head -1)
  python tools/step_timeline.py $f > $O/step_timeline_$tag.txt 2>&1; head -12 $O/step_timeline_$tag.txt
done
for lh in 0 32; do
  for cfg in C3 R3; do
    step "bench lh$lh $cfg"
    NPGX_LONG_HEAD=$lh NPGX_ELF_DEVICE=0 timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_lh${lh}_$cfg.log 2>&1 || { tail -5 $O/bench_lh${lh}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_lh${lh}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('lh$lh $cfg', d['ms_per_step'], 'align', s['ms_stage']['align_batch'], 'af', s['ms_stage']['anchor_finder'])"
  done
done
step done
