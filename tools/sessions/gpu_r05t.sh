#!/bin/bash
# round 5: where a C3 job's cycles go (the profiling build's phase counters), the C3 / R3 / C5 lines
# with fast_run one row at a time (the new default)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05t
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "analyze prof C3"
NPGX_ELF_DEVICE=0 NPGX_PROFILE=1 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C3 > $O/analyze_C3_prof.txt 2>&1 || { tail -5 $O/analyze_C3_prof.txt; exit 1; }
grep -E "phase cycles|fit cycles|cycles per column|top job phases" $O/analyze_C3_prof.txt | head -8
for cfg in C3 R3 C5; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'])"
done
step done
