#!/bin/bash
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04c
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_similar_aligner_gpu.py tests/test_block_build_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "== ab twins C3 $(date +%T)"
tools/gpu_ab_env.sh r04c NPGX_TWINS 0 -1 --config C3 --steps 10 --warmup 3 || exit 1
echo "== ab twins C5 $(date +%T)"
tools/gpu_ab_env.sh r04c NPGX_TWINS 0 -1 --config C5 --steps 3 --warmup 1 || exit 1
echo "== hostprof $(date +%T)"
tools/gpu_hostprof.sh r04c
