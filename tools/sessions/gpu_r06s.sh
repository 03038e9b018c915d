#!/bin/bash
# round 6: AnchorFinder membership table with per-slot fingerprints (the
# occupancy-bit build as libnpge_amd_alt.so; both builds with the
# ExtendLoopFast launch fusions: long-block hash in k_dt_hash_w, Pipe state +
# MoveUnchanged test, OU padding + fragment copies, OU conflict lists +
# priority-ordered lists): parity, A/B at 4 and 8 slots per hash on C3, one
# A/B at C5
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06s
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest af"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_anchor_device_gpu.py tests/test_fullsize_gpu.py tests/test_elf_device_gpu.py tests/test_block_build_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sl in 4 8; do
  step "fp (new) vs occupancy bit (alt), $sl slots, C3"
  NPGX_AF_TABLE_SLOTS=$sl timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config C3 --no-pairs-line > $O/ab_c3_s$sl.txt 2>&1 || { tail -5 $O/ab_c3_s$sl.txt; exit 1; }
  cut -c1-120 $O/ab_c3_s$sl.txt
done
step "fp vs occupancy bit, 8 slots, C5"
NPGX_AF_TABLE_SLOTS=8 timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 1 --config C5 --steps 5 --no-pairs-line > $O/ab_c5_s8.txt 2>&1 || { tail -5 $O/ab_c5_s8.txt; exit 1; }
cut -c1-120 $O/ab_c5_s8.txt
step done
