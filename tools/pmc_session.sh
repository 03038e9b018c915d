#!/bin/bash
# PMC passes over a short bench run (counters collected on their own, one
# group per pass: HBM traffic, then wave-state counters).  Run via gpurun.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-pmc}
CFG=${2:-C2}
mkdir -p gpurun_out
cd /tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | cut -d' ' -f1)
  echo "== pass $name"; date
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_$name -o run -- python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_$name.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/${TAG}_$name.log; exit $rc; }
done
exit 0
