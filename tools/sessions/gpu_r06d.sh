#!/bin/bash
# round 6: unsplit twins (each unsplit job's rows walked reversed beside it)
# and 2 waves per SIMD: aligner parity, full-size C2/C3 parity, A/B of the twins
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06d
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest aligner + device loop"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_elf_device_gpu.py tests/test_block_build_gpu.py > $O/pytest_a.log 2>&1 || { tail -30 $O/pytest_a.log; exit 1; }
tail -2 $O/pytest_a.log
step "pytest fullsize C2/C3"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_fullsize_gpu.py > $O/pytest_full.log 2>&1 || { tail -30 $O/pytest_full.log; exit 1; }
tail -2 $O/pytest_full.log
for cfg in C3 C2 R3; do
  step "ab $cfg"
  timeout -k 10 900 tools/gpu_ab_env.sh r06d NPGX_UTWINS 0 3 --config $cfg --steps 10 --warmup 3 || exit 1
done
step done
