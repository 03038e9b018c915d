#!/bin/bash
# round 6: the Bloom epochs add their new bits to P in place (no copy of the
# m/8-byte array after each epoch; libnpge_amd_alt.so copies) and run one
# launch an epoch (collect of epoch e with the first-setter pass of e+1,
# NPGX_AF_EPOCH_FUSE=0: two): parity both ways, A/B at C3 / C5; C5's Filter
# phases (NPGX_FILTER_DEBUG)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06w
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest af"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_anchor_device_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step "pytest af unfused"
NPGX_AF_EPOCH_FUSE=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_fullsize_gpu.py > $O/pytest_unfused.log 2>&1 || { tail -30 $O/pytest_unfused.log; exit 1; }
tail -1 $O/pytest_unfused.log
for cfg in C3 C5; do
  step "epoch fuse A/B $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06w NPGX_AF_EPOCH_FUSE 0 1 --config $cfg --steps 10 --warmup 3 || exit 1
done
for cfg in C3 C5; do
  step "P in place (new) vs copy (alt), $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config $cfg --steps 10 --no-pairs-line > $O/ab_pinplace_$cfg.txt 2>&1 || { tail -5 $O/ab_pinplace_$cfg.txt; exit 1; }
  cut -c1-140 $O/ab_pinplace_$cfg.txt
done
step "C5 filter phases"
NPGX_FILTER_DEBUG=1 timeout -k 10 300 python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/c5_filter_debug.log 2> $O/c5_filter_debug.err || { tail -5 $O/c5_filter_debug.err; exit 1; }
grep -i filter $O/c5_filter_debug.err | tail -4
step done
