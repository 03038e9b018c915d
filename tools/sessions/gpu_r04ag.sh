#!/bin/bash
# AnchorLoop parity + C2/C3 lines and the C3 adding-loop totals
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04ag
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_anchor_loop_full_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
for cfg in C2 C3; do
  NPGX_AL_DEBUG=1 timeout -k 10 400 python bench.py --config $cfg --anchor-loop full --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_al.log 2> $O/al_debug_$cfg.txt || { tail -5 $O/al_debug_$cfg.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}_al.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print('$cfg', d['value'], d['ms_per_step'], l.get('adding_loop_rounds'), json.dumps(l['ms_loop']))"
done
