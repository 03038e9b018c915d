#!/bin/bash
# round 6: C5 is 210 ms a step against 179 in round 5: the aligner's waves per
# SIMD (2, this round, vs 4: libnpge_amd_alt.so), the unsplit twins and the
# anchors on the device, A/B at C5 (and C3 for the waves)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06t
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "waves 2 (new) vs 4 (alt), C5"
timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config C5 --steps 5 --no-pairs-line > $O/ab_c5_w4.txt 2>&1 || { tail -5 $O/ab_c5_w4.txt; exit 1; }
cut -c1-160 $O/ab_c5_w4.txt
for vv in NPGX_UTWINS:3 NPGX_ANCHOR_DEVICE:1 NPGX_LONG_LDS:1; do
  v=${vv%%:*}; on=${vv##*:}
  step "$v A/B C5"
  timeout -k 10 600 tools/gpu_ab_env.sh r06t $v 0 $on --config C5 --steps 5 --warmup 2 || exit 1
done
step "waves 2 (new) vs 4 (alt), C3"
timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config C3 --no-pairs-line > $O/ab_c3_w4.txt 2>&1 || { tail -5 $O/ab_c3_w4.txt; exit 1; }
cut -c1-160 $O/ab_c3_w4.txt
step done
