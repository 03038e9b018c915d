#!/bin/bash
# round 6: host phases of C3's Filter and AnchorFinder (NPGX_FILTER_DEBUG,
# NPGX_AF_DEBUG) on the final code
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06ab
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "C3 debug phases"
NPGX_FILTER_DEBUG=1 NPGX_AF_DEBUG=1 timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/c3_debug.log 2> $O/c3_debug.err || { tail -5 $O/c3_debug.err; exit 1; }
tail -6 $O/c3_debug.err | cut -c1-250
step done
