#!/bin/bash
# round 6: the 4-wave threshold of the aligner (NPGX_SA_MANY_AT: 2048 tasks,
# default, vs never) at C2 (3-row jobs), C5 and the C4 pair job; the
# AnchorFinder membership table's second bit array (libnpge_amd_alt.so: one
# bit array, and P copied after each Bloom epoch) with its parity tests; the
# new build also adds each epoch's Bloom bits to P in place
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06v
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest af"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_anchor_device_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C5; do
  step "occ2 (new) vs one bit array (alt), $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config $cfg --steps 10 --no-pairs-line > $O/ab_occ2_$cfg.txt 2>&1 || { tail -5 $O/ab_occ2_$cfg.txt; exit 1; }
  cut -c1-140 $O/ab_occ2_$cfg.txt
done
for cfg in C2 C5; do
  step "threshold A/B $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06v NPGX_SA_MANY_AT 1000000000 2048 --config $cfg --steps 10 --warmup 3 || exit 1
done
for rep in 1 2; do
  for v in 1000000000 2048; do
    step "pairs NPGX_SA_MANY_AT=$v"
    NPGX_SA_MANY_AT=$v timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_${v}_$rep.log 2>&1 || { tail -5 $O/pairs_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/pairs_${v}_$rep.log').read().strip().splitlines()[-1]); print('pairs', '$v', d['value'], d['ms_per_step'])"
  done
done
step done
