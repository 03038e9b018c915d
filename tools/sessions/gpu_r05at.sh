#!/bin/bash
# round 5: where the host time of C3 + AnchorLoopFast goes (SIGPROF samples of
# the library; the step is 72 % host by the kernel trace, gpurun_out/r05ar)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05at
mkdir -p $O
echo "== hostprof C3 alf $(date +%T)"
timeout -k 10 400 python tools/host_profile.py C3 5 alf > $O/host_C3_alf.txt 2>&1 || { tail -5 $O/host_C3_alf.txt; exit 1; }
head -60 $O/host_C3_alf.txt
echo "== done $(date +%T)"
