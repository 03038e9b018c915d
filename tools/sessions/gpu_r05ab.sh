#!/bin/bash
# round 5: R3 with AnchorLoopFast (the wide aligner's share) and the wide-aligner batch bench
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ab
mkdir -p $O
echo "== r3 alf $(date +%T)"
timeout -k 10 400 python bench.py --config R3 --anchor-loop --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_R3_alf.log 2>&1 || { tail -5 $O/bench_R3_alf.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_R3_alf.log').read().strip().splitlines()[-1]); s=d['last_step']; print(d['ms_per_step'], s.get('anchor_loop',{}).get('ms_loop'), [(k['name'], round(k['ms'],1)) for k in d.get('kernels_last_step',[])])"
echo "== bench_wide $(date +%T)"
timeout -k 10 400 python tools/bench_wide.py > $O/bench_wide.log 2>&1 || { tail -5 $O/bench_wide.log; exit 1; }
tail -12 $O/bench_wide.log
echo "== done $(date +%T)"
