#!/bin/bash
# round 5: LDS per aligner slot (rows staged in LDS instead of read from global memory) -- the cap on
# resident slots per CU (NPGX_SA_PER_CU_MAX) at C3 / R3 / C5
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aa
mkdir -p $O
for pc in 16 4 2 1; do
  for cfg in C3 R3 C5; do
    echo "== pc$pc $cfg $(date +%T)"
    NPGX_SA_PER_CU_MAX=$pc timeout -k 10 300 python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/bench_pc${pc}_$cfg.log 2>&1 || { tail -5 $O/bench_pc${pc}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_pc${pc}_$cfg.log').read().strip().splitlines()[-1]); print('pc$pc $cfg', d['ms_per_step'])"
  done
done
echo "== done $(date +%T)"
