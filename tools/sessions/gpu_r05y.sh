#!/bin/bash
# round 5: the asynchronous aligner's batch preparation per phase at C2 / C3 (device loop)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05y
mkdir -p $O
for cfg in C2 C3; do
  echo "== prep $cfg $(date +%T)"
  NPGX_PREP_DEBUG=1 timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prep_$cfg.log 2> $O/prep_$cfg.err || { tail -5 $O/prep_$cfg.err; exit 1; }
  grep "align_device" $O/prep_$cfg.err | tail -10
done
echo "== done $(date +%T)"
