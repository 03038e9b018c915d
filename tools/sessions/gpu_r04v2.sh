#!/bin/bash
# round-4 perf evidence: C2/C4/C5/anchor-loop benches, C3 rocprof + PMC
# passes (tools/round_end.sh perf), then the AnchorLoop lines (C2, C3) with
# their round costs and the oracle's AnchorLoop on C2 on this host
set -o pipefail
R=$(pwd)
TAG=${1:-r04v}
O=$R/gpurun_out/$TAG
mkdir -p $O
echo "== pytest anchor loop $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_anchor_loop_full_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest_al.log 2>&1 || { tail -40 $O/pytest_al.log | cut -c1-300; exit 1; }
tail -1 $O/pytest_al.log
tools/round_end.sh $TAG perf || exit 1
for cfg in C2 C3; do
  echo "== bench $cfg AnchorLoop $(date +%T)"
  timeout -k 10 400 python bench.py --config $cfg --anchor-loop full --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_al.log 2>&1 || { tail -5 $O/bench_${cfg}_al.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}_al.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print(d['value'], d['ms_per_step'], l.get('adding_loop_rounds'), json.dumps(l['ms_loop']))"
done
NPGX_AL_DEBUG=1 timeout -k 10 300 python bench.py --config C2 --anchor-loop full --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/bench_C2_al_dbg.log 2> $O/al_debug_C2.txt || { tail -5 $O/al_debug_C2.txt; exit 1; }
grep "24[0-9][0-9][0-9] blocks in" $O/al_debug_C2.txt
echo "== cpu AnchorLoop C2 $(date +%T)"
timeout -k 10 300 python tools/cpu_anchor_loop.py C2 > $O/cpu_anchor_loop_C2.json 2>&1 || { tail -5 $O/cpu_anchor_loop_C2.json; exit 1; }
cat $O/cpu_anchor_loop_C2.json | cut -c1-300
