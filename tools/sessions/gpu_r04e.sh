#!/bin/bash
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04e
mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_block_build_gpu.py tests/test_fullsize_gpu.py tests/test_pairs_gpu.py tests/test_script_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "== ab fe_small C3 $(date +%T)"
tools/gpu_ab_env.sh r04e NPGX_FE_SMALL 0 1 --config C3 --steps 10 --warmup 3 || exit 1
echo "== ab twins C3 $(date +%T)"
tools/gpu_ab_env.sh r04e NPGX_TWINS 0 -1 --config C3 --steps 10 --warmup 3 || exit 1
echo "== ab fe_small pairs $(date +%T)"
tools/gpu_ab_env.sh r04e NPGX_FE_SMALL 0 1 --mode pairs --pairs 96 --steps 2 --warmup 1 || exit 1
for cfg in C3 C4:pair; do
  echo "== hostprof $cfg $(date +%T)"
  timeout -k 10 300 python tools/host_profile.py $cfg 150 > $O/host_$cfg.txt 2>&1 || { tail -5 $O/host_$cfg.txt; exit 1; }
  head -25 $O/host_$cfg.txt
done
