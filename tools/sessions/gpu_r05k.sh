#!/bin/bash
# round 5: why R3's late flank jobs re-run (retry diagnostics, host loop), and the pair job's
# regression: device loop vs host loop, prefix search on / off
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05k
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "r3 retry debug"
NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 300 python bench.py --config R3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3_retry.log 2> $O/r3_retry.err || { tail -5 $O/r3_retry.err; exit 1; }
grep -c "retry job" $O/r3_retry.err; grep "retry job" $O/r3_retry.err | head -30
for v in dev128:1:128 host128:0:128 dev0:1:0; do
  IFS=: read tag dev lh <<< "$v"
  step "pairs $tag"
  NPGX_ELF_DEVICE=$dev NPGX_LONG_HEAD=$lh timeout -k 10 500 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$tag.log 2>&1 || { tail -5 $O/pairs_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], {k: v for k, v in d.items() if k.startswith('mean_pair')})"
done
step done
