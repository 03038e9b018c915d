#!/bin/bash
# host phase times of a C3 step (AnchorFinder host, aligner prep) to stderr
set -o pipefail
mkdir -p gpurun_out/hd
NPGX_AF_DEBUG=1 NPGX_PREP_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/hd/c3.json 2> gpurun_out/hd/c3.err
rc=$?; tail -3 gpurun_out/hd/c3.err | cut -c1-300; exit $rc
