#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r04f
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_block_build_gpu.py tests/test_fullsize_gpu.py tests/test_pairs_gpu.py tests/test_similar_aligner_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "== ab timers C3 $(date +%T)"
tools/gpu_ab_env.sh r04f NPGX_TIMERS 1 0 --config C3 --steps 10 --warmup 3 || exit 1
echo "== ab fe_small C2 $(date +%T)"
tools/gpu_ab_env.sh r04f NPGX_FE_SMALL 0 1 --config C2 --steps 10 --warmup 3 || exit 1
echo "== ab fe_small pairs $(date +%T)"
tools/gpu_ab_env.sh r04f NPGX_FE_SMALL 0 1 --mode pairs --pairs 96 --steps 2 --warmup 1 || exit 1
echo "== hip trace C3 $(date +%T)"
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d $O/hip -o run -- python3 $R/bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/hip.log 2>&1 || { tail -5 $O/hip.log; exit 1; }
cd $R
ls $O/hip/*/ 2>/dev/null | head; f=$(ls $O/hip/*/*hip_api_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -25 "$f" | cut -c1-160
