#!/bin/bash
# round 6: the Bloom epochs add their new bits to P in place (no copy of the
# m/8-byte array after each epoch; libnpge_amd_alt.so copies): parity, A/B at
# C3 / C5
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06w
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest af"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_anchor_device_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C5; do
  step "P in place (new) vs copy (alt), $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 3 --config $cfg --steps 10 --no-pairs-line > $O/ab_pinplace_$cfg.txt 2>&1 || { tail -5 $O/ab_pinplace_$cfg.txt; exit 1; }
  cut -c1-140 $O/ab_pinplace_$cfg.txt
done
step done
