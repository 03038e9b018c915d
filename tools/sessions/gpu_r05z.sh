#!/bin/bash
# round 5: where k_align_jobs / k_align_sub waves wait at C3 (SQ counters, two passes)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05z
mkdir -p $O
cd /tmp
echo "== pass1 $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
echo "== pass2 $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
echo "== done $(date +%T)"
