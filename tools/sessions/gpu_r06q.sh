#!/bin/bash
# round 6: OverlaplessUnion of small tables (one-workgroup block sort with the
# fragment copies, priorities and pads; fused conflict lists + admission):
# parity (both paths), NPGX_OU_SMALL A/B at C3 / C2, a C3 kernel trace;
# AnchorFinder counts of the groups the cut can keep only (NPGX_AF_COUNT_ALL A/B)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06q
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest ou"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_fullsize_gpu.py tests/test_block_build_gpu.py tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_anchor_device_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C2; do
  step "ou small A/B $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06q NPGX_OU_SMALL 0 1 --config $cfg --steps 10 --warmup 3 || exit 1
done
step "af count A/B C3"
timeout -k 10 600 tools/gpu_ab_env.sh r06q NPGX_AF_COUNT_ALL 1 0 --config C3 --steps 10 --warmup 3 || exit 1
step "rocprof C3"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python $R/bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
cd $R
step done
