#!/bin/bash
# round 5: the pair job with the prefix search -- scratch limit raised (HSA_SCRATCH_SINGLE_LIMIT) and
# find_word_long inlined (488 B of scratch instead of 664); C3 / R3 for the inlined build
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05o
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for v in curlim:libnpge_amd.so:4294967296 inl:libnpge_amd_inl.so: inllim:libnpge_amd_inl.so:4294967296; do
  IFS=: read tag lib lim <<< "$v"
  step "pairs $tag"
  if [ -n "$lim" ]; then export HSA_SCRATCH_SINGLE_LIMIT=$lim; else unset HSA_SCRATCH_SINGLE_LIMIT; fi
  NPGX_LIB=$lib NPGX_ELF_DEVICE=0 timeout -k 10 500 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$tag.log 2>&1 || { tail -5 $O/pairs_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$tag.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag', d['value'], d['ms_per_step'], 'af', s['mean_pair_ms']['anchor_finder'], 'align', s['mean_pair_ms_align'])"
done
unset HSA_SCRATCH_SINGLE_LIMIT
for cfg in C3 R3; do
  step "inl $cfg"
  NPGX_LIB=libnpge_amd_inl.so timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_inl_$cfg.log 2>&1 || { tail -5 $O/bench_inl_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_inl_$cfg.log').read().strip().splitlines()[-1]); print('inl $cfg', d['ms_per_step'])"
done
step done
