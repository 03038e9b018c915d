#!/bin/bash
# C3 diagnostics in one call: aligner split/sub critical paths, then the host-side sampling profile
set -o pipefail
mkdir -p gpurun_out/sd gpurun_out/hp
#timeout -k 10 200 python -u tools/split_stats.py C3 > gpurun_out/sd/c3.out 2> gpurun_out/sd/c3.err
echo split_stats exit $?
timeout -k 10 240 python -u tools/host_profile.py C3 80 > gpurun_out/hp/out_C3.txt 2>&1
echo host_profile exit $?
