#!/bin/bash
# A/B of two library builds at C3 and C2 on one box (diagnostic):
#   tools/ab_c3.sh <alt .so in npge_amd/> [rounds]
ALT=$1; N=${2:-2}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for cfg in C3 C2; do
    for v in new alt; do
      if [ $v = alt ]; then export NPGX_LIB=$ALT; else unset NPGX_LIB; fi
      st=4; [ $cfg = C2 ] && st=15
      timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
      python - "$v" "$cfg" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
s = d["last_step"]["ms_stage"]
print(sys.argv[2], sys.argv[1], d["ms_per_step"], "align=%.2f" % s["align_batch"], "kwait=%.2f" % s["align_kernel_wait"])
PY
    done
  done
done
