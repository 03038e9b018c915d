#!/bin/bash
# round 5: where k_align_jobs' writes come from: FETCH_SIZE / WRITE_SIZE passes
# at C3 with the prefix word search (default) and without it (NPGX_LONG_HEAD=0)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05az
mkdir -p $O
cd /tmp
for v in lh128: lh0:0; do
  tag=${v%%:*}; lh=${v#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $tag $c $(date +%T)"
    if [ -n "$lh" ]; then export NPGX_LONG_HEAD=$lh; else unset NPGX_LONG_HEAD; fi
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${tag}_$c -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/${tag}_$c.log 2>&1 || { tail -5 $O/${tag}_$c.log; exit 1; }
  done
done
unset NPGX_LONG_HEAD
echo "== done $(date +%T)"
