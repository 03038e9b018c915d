#!/bin/bash
# round 5: AnchorFinder slot counts on / off (C3, C5), the R3 kernel breakdown, AnchorLoopFast at
# C3 / C4 and the pair job with the device loop
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05j
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
b() {  # tag cfg extra-args -- env...
  local tag=$1 cfg=$2 extra=$3; shift 3
  env "$@" timeout -k 10 400 python bench.py --config $cfg $extra --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_$cfg.log 2>&1 || { tail -5 $O/bench_${tag}_$cfg.log; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_${tag}_$cfg.log').read().strip().splitlines()[-1]); s=d.get('last_step',{}); print('$tag $cfg', d['ms_per_step'], d['value'], 'af', s.get('ms_stage',{}).get('anchor_finder'))"
}
for sc in 0 1; do
  for cfg in C3 C5; do
    step "af slot$sc $cfg"; b slot$sc $cfg "--steps 5 --warmup 2" NPGX_AF_SLOT_COUNT=$sc || exit 1
  done
done
step "alf C3"; b alf C3 "--anchor-loop --steps 3 --warmup 1" NPGX_X=1 || exit 1
step "alf C4"; b alf C4 "--anchor-loop --steps 3 --warmup 1" NPGX_X=1 || exit 1
step "rocprof R3"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r3 -o run -- python3 $R/bench.py --config R3 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_r3.log 2>&1 || { tail -5 $O/prof_r3.log; exit 1; }
cd $R
step "pairs C4"
timeout -k 10 500 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_pairs.log 2>&1 || { tail -5 $O/bench_pairs.log; exit 1; }
tail -1 $O/bench_pairs.log | cut -c1-400
step done
