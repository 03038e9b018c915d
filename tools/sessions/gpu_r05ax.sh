#!/bin/bash
# round 5: AnchorLoopFast phase ticks at C3 (NPGX_LOOP_DEBUG) and the AnchorFinder host phases (NPGX_AF_DEBUG)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ax
mkdir -p $O
echo "== loop debug $(date +%T)"
NPGX_LOOP_DEBUG=1 NPGX_AF_DEBUG=1 timeout -k 10 300 python bench.py --config C3 --anchor-loop --steps 2 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/c3alf.log 2> $O/c3alf.err || { tail -5 $O/c3alf.err; exit 1; }
tail -1 $O/c3alf.log | cut -c1-150
tail -60 $O/c3alf.err
echo "== done $(date +%T)"
