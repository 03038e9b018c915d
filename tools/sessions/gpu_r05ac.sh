#!/bin/bash
# round 5: why R3 + AnchorLoopFast re-runs aligner jobs (reason codes, host loop)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ac
mkdir -p $O
echo "== r3 alf retries $(date +%T)"
NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 400 python bench.py --config R3 --anchor-loop --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3alf.log 2> $O/r3alf.err || { tail -5 $O/r3alf.err; exit 1; }
echo "retried: $(grep -c 'retry job' $O/r3alf.err)"
grep "retry job" $O/r3alf.err | awk '{print $NF}' | sort | uniq -c
grep "retry job" $O/r3alf.err | sort -t' ' -k7 -n -r | head -20
echo "== done $(date +%T)"
