#!/bin/bash
# round 5: prefix word search (find_word_long) -- aligner parity, then C3 / R3 per-job costs old vs new
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05b
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py > $O/pytest_sa.log 2>&1 || { tail -30 $O/pytest_sa.log; exit 1; }
tail -3 $O/pytest_sa.log
for c in C3 R3; do
  for h in 0 32; do
    step "analyze $c head $h"
    NPGX_LONG_HEAD=$h NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py $c > $O/analyze_${c}_h$h.txt 2>&1 || { tail -5 $O/analyze_${c}_h$h.txt; exit 1; }
    grep -E "^rep 4|fit cycles|jobs .* total" $O/analyze_${c}_h$h.txt
  done
done
step bench
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_C3.log 2>&1 || { tail -5 $O/bench_C3.log; exit 1; }
tail -1 $O/bench_C3.log | cut -c1-400
timeout -k 10 300 python bench.py --config R3 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_R3.log 2>&1 || { tail -5 $O/bench_R3.log; exit 1; }
tail -1 $O/bench_R3.log | cut -c1-400
step elf_device
NPGX_LIB=libnpge_amd_next.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py > $O/pytest_elf.log 2>&1 || { tail -40 $O/pytest_elf.log; exit 1; }
tail -3 $O/pytest_elf.log
NPGX_LIB=libnpge_amd_next.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_C3_next.log 2>&1 || { tail -5 $O/bench_C3_next.log; exit 1; }
tail -1 $O/bench_C3_next.log | cut -c1-600
step done
