#!/bin/bash
# round 5: full-suffix segment rooms for split jobs (NPGX_SEG_FULL_MB, default 64; 0 = round-4 rooms):
# aligner and repeat parity, R3 retries and step time, C3 / C5 lines
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05m
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for mb in 0 64; do
  step "r3 retries seg_full $mb"
  NPGX_SEG_FULL_MB=$mb NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 300 python bench.py --config R3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3_retry_$mb.log 2> $O/r3_retry_$mb.err || { tail -5 $O/r3_retry_$mb.err; exit 1; }
  echo "retried jobs: $(grep -c 'retry job' $O/r3_retry_$mb.err)"
  for cfg in R3 C3 C5; do
    step "bench seg_full $mb $cfg"
    NPGX_SEG_FULL_MB=$mb timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/bench_${mb}_$cfg.log 2>&1 || { tail -5 $O/bench_${mb}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${mb}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$mb $cfg', d['ms_per_step'], [(k['name'], round(k['ms'], 2)) for k in d.get('kernels_last_step', [])])"
  done
done
step done
# the pair job's kernels, round-4 library vs the current one (host loop), 64 pairs
export TMPDIR=/tmp
for v in r04:libnpge_amd_r04.so:0 cur:libnpge_amd.so:0; do
  IFS=: read tag lib dev <<< "$v"
  step "rocprof pairs $tag"
  cd /tmp
  NPGX_LIB=$lib NPGX_ELF_DEVICE=$dev timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pairs_$tag -o run -- python3 $R/bench.py --mode pairs --config C4 --pairs 64 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_pairs_$tag.log 2>&1 || { tail -5 $O/prof_pairs_$tag.log; exit 1; }
  cd $R
  tail -1 $O/prof_pairs_$tag.log | cut -c1-200
done
step done2
