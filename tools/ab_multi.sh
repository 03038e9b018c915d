#!/bin/bash
# bench.py at C2 and C3 for several library builds in npge_amd/ (diagnostic):
#   tools/ab_multi.sh "default libnpge_amd_x.so ..." [rounds]
LIBS=$1; N=${2:-2}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for cfg in C2 C3; do
    for v in $LIBS; do
      if [ $v = default ]; then unset NPGX_LIB; else export NPGX_LIB=$v; fi
      st=4; [ $cfg = C2 ] && st=15
      timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline > gpurun_out/abm.log 2>&1 || { tail -5 gpurun_out/abm.log; exit 1; }
      python - "$v" "$cfg" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abm.log").read().strip().splitlines()[-1])
s = d["last_step"]["ms_stage"]
print(sys.argv[2], sys.argv[1], d["ms_per_step"], "align=%.2f" % s["align_batch"], "kwait=%.2f" % s["align_kernel_wait"])
PY
    done
  done
done
