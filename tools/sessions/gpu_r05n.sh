#!/bin/bash
# round 5: the pair job against round 4 with the prefix search compiled out (its call costs
# k_align_jobs 664 B of scratch against 312 B), and why R3's split jobs re-run (reason codes)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05n
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "r3 retry reasons"
NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 300 python bench.py --config R3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3_retry.log 2> $O/r3_retry.err || { tail -5 $O/r3_retry.err; exit 1; }
grep "retry job" $O/r3_retry.err | head -20
for v in nolong:libnpge_amd_nolong.so nolongfr1:libnpge_amd_nolongfr1.so cur:libnpge_amd.so r04:libnpge_amd_r04.so; do
  IFS=: read tag lib <<< "$v"
  step "pairs $tag"
  NPGX_LIB=$lib NPGX_ELF_DEVICE=0 timeout -k 10 500 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$tag.log 2>&1 || { tail -5 $O/pairs_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$tag.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag', d['value'], d['ms_per_step'], 'af', s['mean_pair_ms']['anchor_finder'], 'align', s['mean_pair_ms_align'], 'host', s['mean_pair_ms_host'])"
done
for cfg in C3 R3; do
  step "nolong $cfg"
  NPGX_LIB=libnpge_amd_nolong.so timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_nolong_$cfg.log 2>&1 || { tail -5 $O/bench_nolong_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_nolong_$cfg.log').read().strip().splitlines()[-1]); print('nolong $cfg', d['ms_per_step'])"
done
step done
