#!/bin/bash
# the repeat-rich R3 set (C3-shaped, planted IS-like families): DraftPangenome
# line and DraftPangenome -> AnchorLoopFast line
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04aj
mkdir -p $O
timeout -k 10 300 python bench.py --config R3 --steps 5 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_R3.log 2>&1 || { tail -5 $O/bench_R3.log; exit 1; }
tail -1 $O/bench_R3.log | cut -c1-200
timeout -k 10 400 python bench.py --config R3 --anchor-loop fast --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_R3_alf.log 2>&1 || { tail -5 $O/bench_R3_alf.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_R3_alf.log').read().strip().splitlines()[-1]); print('R3 alf', d['value'], d['ms_per_step'], json.dumps(d['last_step'].get('anchor_loop', {}).get('ms_loop')))"
