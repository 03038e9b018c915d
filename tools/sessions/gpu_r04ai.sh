#!/bin/bash
# GPU occupancy of the pair job with the round-4 defaults (16 workers, 20 hardware queues)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r04ai
mkdir -p $O
cd /tmp
GPU_MAX_HW_QUEUES=20 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_pairs -o run -- python3 $R/bench.py --mode pairs --steps 1 --warmup 1 --no-cpu-baseline > $O/pairs.log 2>&1 || { tail -5 $O/pairs.log; exit 1; }
cd $R
python3 tools/pairs_busy.py $O/prof_pairs/run_kernel_trace.csv > $O/pairs_busy.txt 2>&1
head -12 $O/pairs_busy.txt
