#!/bin/bash
# round 5: HIP API time of C3 + AnchorLoopFast (which runtime calls hold the
# host while the GPU idles: allocations, frees, copies, waits)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05au
mkdir -p $O
cd /tmp
echo "== rocprof hip api C3 alf $(date +%T)"
timeout -k 10 400 rocprofv3 --hip-runtime-trace --stats --output-format csv -d $O/api_c3_alf -o run -- python3 $R/bench.py --config C3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/api_c3_alf.log 2>&1 || { tail -5 $O/api_c3_alf.log; exit 1; }
tail -1 $O/api_c3_alf.log | cut -c1-200
ls $O/api_c3_alf
echo "== done $(date +%T)"
