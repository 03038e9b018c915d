#!/bin/bash
# AnchorLoop bench lines (C2, C3; fast vs full) and a rocprof kernel summary
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r04n
mkdir -p $O
for cfg in C2 C3; do
  for pipe in fast full; do
    echo "== bench $cfg $pipe $(date +%T)"
    timeout -k 10 400 python bench.py --config $cfg --anchor-loop $pipe --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_$pipe.log 2>&1 || { tail -5 $O/bench_${cfg}_$pipe.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${cfg}_$pipe.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print(d['value'], d['ms_per_step'], json.dumps({k: v for k, v in (l or {}).items() if not isinstance(v, dict)}))"
  done
done
echo "== rocprof C3 full $(date +%T)"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_full -o run -- python3 $R/bench.py --config C3 --anchor-loop full --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3_full.log 2>&1 || { tail -5 $O/prof_c3_full.log; exit 1; }
head -15 $O/prof_c3_full/run_kernel_stats.csv | cut -d, -f1-4
