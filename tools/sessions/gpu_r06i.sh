#!/bin/bash
# round 6: host phases between the AnchorFinder and the first decode (C3,
# C2), and a C2 kernel trace
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06i
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for cfg in C3 C2; do
  step "debug $cfg"
  NPGX_AF_DEBUG=1 NPGX_BB_DEBUG=1 timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/dbg_$cfg.log 2>&1 || { tail -5 $O/dbg_$cfg.log; exit 1; }
  grep -E "af host|draft:" $O/dbg_$cfg.log | tail -4
done
cd /tmp
step "rocprof C2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
python3 $R/tools/step_timeline.py $O/prof_c2/run_kernel_trace.csv | head -12
step done
