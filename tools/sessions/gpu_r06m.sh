#!/bin/bash
# round 6: 8 waves per sync-state search, twins filling the last 256-task
# step of every launch -- parity, the twins A/B; AnchorLoopFast with the
# buffer cache
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06m
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_elf_device_gpu.py tests/test_repeats_gpu.py tests/test_fullsize_gpu.py tests/test_anchor_device_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 R3; do
  step "utwins $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06m NPGX_UTWINS 0 3 --config $cfg --steps 10 --warmup 3 || exit 1
done
step "alf buf cache"
timeout -k 10 600 tools/gpu_ab_env.sh r06m NPGX_BUF_CACHE 0 1 --config C3 --anchor-loop --steps 3 --warmup 1 || exit 1
step done
