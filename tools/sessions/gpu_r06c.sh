#!/bin/bash
# round 6: the aligner kernels at 2 and 3 waves per SIMD (no scratch spills)
# against the default 4: C3, C2, R3 and the pair job, alternating builds
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06c
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for cfg in C3 R3 C2; do
  step "ab $cfg"
  for lib in libnpge_amd_w2.so libnpge_amd_w3.so; do
    timeout -k 10 600 tools/ab_bench.sh $lib 2 --config $cfg --no-pairs-line > $O/ab_${cfg}_$lib.txt 2>&1 || { tail -5 $O/ab_${cfg}_$lib.txt; exit 1; }
    echo $lib; cut -c1-200 $O/ab_${cfg}_$lib.txt
  done
done
for lib in "" libnpge_amd_w2.so; do
  step "pairs $lib"
  NPGX_LIB=$lib timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$lib.log 2>&1 || { tail -5 $O/pairs_$lib.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$lib.log').read().strip().splitlines()[-1]); print('pairs', '$lib', d['value'], d['ms_per_step'])"
done
step done
