#!/bin/bash
# round 6: DraftPangenome's anchors on the device (anchors_to_device) --
# parity, full-size C2/C3, A/B against the host path
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06k
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_device_gpu.py tests/test_elf_device_gpu.py tests/test_block_build_gpu.py tests/test_anchor_finder_gpu.py tests/test_similar_aligner_gpu.py tests/test_fullsize_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
for cfg in C3 C2; do
  step "ab anchors $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06k NPGX_ANCHOR_DEVICE 0 1 --config $cfg --steps 10 --warmup 3 || exit 1
done
step done
step "pairs device loop"
NPGX_PAIR_TUNING='{"long-head": 0, "elf-device": 1}' timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_dev.log 2>&1 || { tail -5 $O/pairs_dev.log; exit 1; }
python -c "import json; d=json.loads(open('$O/pairs_dev.log').read().strip().splitlines()[-1]); print('pairs dev', d['value'], d['ms_per_step'])"
step "pairs host loop"
timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_host.log 2>&1 || { tail -5 $O/pairs_host.log; exit 1; }
python -c "import json; d=json.loads(open('$O/pairs_host.log').read().strip().splitlines()[-1]); print('pairs host', d['value'], d['ms_per_step'])"
step done2
