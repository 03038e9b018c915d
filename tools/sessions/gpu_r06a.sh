#!/bin/bash
# round 6 baseline on this round's box: C3 aligner phase counters (profiling
# build, device loop), the C3 / C2 lines, the pair line with the host and the
# device ExtendLoopFast
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06a
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "elf device tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_buf_cache_gpu.py > $O/pytest_elf.log 2>&1 || { tail -30 $O/pytest_elf.log; exit 1; }
tail -2 $O/pytest_elf.log
step "analyze prof C3"
NPGX_PROFILE=1 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_C3_prof.txt 2>&1 || { tail -5 $O/analyze_C3_prof.txt; exit 1; }
grep -E "phase cycles|fit cycles|cycles per column|top job phases" $O/analyze_C3_prof.txt | head -8
for cfg in C3 C2; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['stage_timeline'])"
done
step "pairs host loop"
timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_pairs_host.log 2>&1 || { tail -5 $O/bench_pairs_host.log; exit 1; }
tail -1 $O/bench_pairs_host.log | cut -c1-400
step "pairs device loop"
NPGX_PAIR_TUNING='{"long-head": 0, "elf-device": 1}' timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_pairs_dev.log 2>&1 || { tail -5 $O/bench_pairs_dev.log; exit 1; }
tail -1 $O/bench_pairs_dev.log | cut -c1-400
step done
