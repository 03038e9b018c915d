#!/bin/bash
# AnchorLoop with settled blocks skipping Align: parity (all sizes), then C2 / C3
# bench lines, with the A/B switch NPGX_AL_ALIGN_ALL=1 (Align every block)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04r
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_anchor_loop_full_gpu.py tests/test_anchor_loop_gpu.py tests/test_align_pipe_gpu.py tests/test_block_build_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
for cfg in C2 C3; do
  for ab in 0 1; do
    echo "== bench $cfg full align_all=$ab $(date +%T)"
    if [ $ab = 1 ]; then export NPGX_AL_ALIGN_ALL=1; else unset NPGX_AL_ALIGN_ALL; fi
    timeout -k 10 400 python bench.py --config $cfg --anchor-loop full --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_$ab.log 2>&1 || { tail -5 $O/bench_${cfg}_$ab.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${cfg}_$ab.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print(d['value'], d['ms_per_step'], json.dumps({k: v for k, v in (l or {}).items() if not isinstance(v, dict)}))"
  done
done
