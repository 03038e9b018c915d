#!/bin/bash
# AnchorLoop phase times (C2, C3)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04s
mkdir -p $O
for cfg in C2 C3; do
  echo "== bench $cfg full $(date +%T)"
  timeout -k 10 400 python bench.py --config $cfg --anchor-loop full --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}.log 2>&1 || { tail -5 $O/bench_${cfg}.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print(d['value'], d['ms_per_step'], l.get('adding_loop_rounds'), json.dumps(l['ms_loop']))"
done
