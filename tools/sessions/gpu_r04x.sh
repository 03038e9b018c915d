#!/bin/bash
# after Filter's all-kept early exit: parity (AnchorLoop, Align pipe, block
# build, anchor loop fast), SmthUnion part times, AnchorLoop C2/C3, default C3 line
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04x
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_anchor_loop_full_gpu.py tests/test_align_pipe_gpu.py tests/test_block_build_gpu.py tests/test_anchor_loop_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
NPGX_AL_DEBUG=1 timeout -k 10 300 python bench.py --config C2 --anchor-loop full --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/bench_C2_al_dbg.log 2> $O/al_debug_C2.txt || { tail -5 $O/al_debug_C2.txt; exit 1; }
grep "24[0-9][0-9][0-9] blocks in" $O/al_debug_C2.txt
for cfg in C2 C3; do
  echo "== bench $cfg AnchorLoop $(date +%T)"
  timeout -k 10 400 python bench.py --config $cfg --anchor-loop full --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_al.log 2>&1 || { tail -5 $O/bench_${cfg}_al.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}_al.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print(d['value'], d['ms_per_step'], l.get('adding_loop_rounds'), json.dumps(l['ms_loop']))"
done
echo "== bench C3 $(date +%T)"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_C3.log 2>&1 || { tail -5 $O/bench_C3.log; exit 1; }
tail -1 $O/bench_C3.log | cut -c1-250
