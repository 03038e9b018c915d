#!/bin/bash
# round 5: the pair job's regression against round 4 -- the round-4 library (built from its commit),
# the current one with the host loop, with the round-4 fast_run order (fr1), without the prefix search
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05l
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for v in r04:libnpge_amd_r04.so:0:0 host:libnpge_amd.so:0:128 fr1:libnpge_amd_fr1.so:0:0 hostlh0:libnpge_amd.so:0:0 dev:libnpge_amd.so:1:128; do
  IFS=: read tag lib dev lh <<< "$v"
  step "pairs $tag"
  NPGX_LIB=$lib NPGX_ELF_DEVICE=$dev NPGX_LONG_HEAD=$lh timeout -k 10 500 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$tag.log 2>&1 || { tail -5 $O/pairs_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$tag.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag', d['value'], d['ms_per_step'], 'af', s['mean_pair_ms']['anchor_finder'], 'align', s['mean_pair_ms_align'], 'host', s['mean_pair_ms_host'])"
done
step done
